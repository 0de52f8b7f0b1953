#!/bin/bash
# round-4 GPU batch 11: config 2 decoder -- is it bound by the lanes' block loads?  Default build vs
# FC_DEC_ABL=8 (every lane reads one of 8 clients' streams: cache-resident loads, same control flow)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for rep in 1 2; do for v in "" _dabl8 _chunk2; do
  echo "== lib$v config2" >> gpurun_out/c2dec.txt
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=6 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -3 >> gpurun_out/c2dec.txt || exit 1
  echo "== lib$v headline" >> gpurun_out/c2dec.txt
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so C=1024 ITERS=3 timeout -k 10 150 python3 tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/c2dec.txt || exit 1
done; done
cat gpurun_out/c2dec.txt
