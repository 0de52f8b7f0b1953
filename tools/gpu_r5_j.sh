#!/bin/bash
# round-5 J: eight-tile tickets in 8-wave workgroups -- super-tile parity tests, then
# k_encode2 at NT = 4 / 8 (1024 x 25 M, stochastic and uniform)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_supertile.py tests/test_gpu_chain.py > gpurun_out/r5j_tests.txt 2>&1 || { tail -30 gpurun_out/r5j_tests.txt; exit 1; }
tail -2 gpurun_out/r5j_tests.txt
O=gpurun_out/r5j.txt
: > $O
for m in 1 0; do
  for nt in 4 8; do
    FEDCODEC_ENC_NT=$nt MODE=$m CAP=0.6 REPS=5 timeout -k 10 240 python3 tools/enc_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/NT=$nt /" >> $O || exit 1
  done
done
cat $O
timeout -k 10 900 python3 bench.py > gpurun_out/r5j_bench.json 2> gpurun_out/r5j_bench.err || { tail -20 gpurun_out/r5j_bench.err; exit 1; }
head -c 600 gpurun_out/r5j_bench.json
