#!/bin/bash
# round-4 GPU batch 14: the guessed parse on untracked batch-point loads (FC_IDX_ASYNC=1; slow paths drain the
# reader first) -- bare-decode tests on that build, then the rebuild timing of both builds
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
A=$PWD/federated_amd/libfedcodec_idxasync.so
FEDCODEC_LIB=$A timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_bare_decode.py tests/test_gpu_large_p.py > gpurun_out/idxasync_tests.log 2>&1 || { tail -30 gpurun_out/idxasync_tests.log; exit 1; }
tail -1 gpurun_out/idxasync_tests.log
for v in "$A" "$PWD/federated_amd/libfedcodec.so"; do
  echo "== $v"
  FEDCODEC_LIB=$v timeout -k 10 200 python3 tools/index_bench.py 2>&1 | grep -v amdgpu.ids || exit 2
done
for rep in 1 2; do
  C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=6 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -2
  C=1024 ITERS=3 timeout -k 10 150 python3 tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -1
done
