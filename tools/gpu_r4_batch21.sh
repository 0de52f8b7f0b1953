#!/bin/bash
# round-4 GPU batch 21: decoder refill by selects (FC_DEC_SEL_REFILL=1) at config 2 and the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
S=$PWD/federated_amd/libfedcodec_selrefill.so
FEDCODEC_LIB=$S timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_quarters.py tests/test_gpu_configs.py > gpurun_out/sel_tests.log 2>&1 || { tail -30 gpurun_out/sel_tests.log; exit 1; }
tail -1 gpurun_out/sel_tests.log
for rep in 1 2; do for v in "$S" "$PWD/federated_amd/libfedcodec.so"; do
  echo "== $(basename $v)"
  FEDCODEC_LIB=$v C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=6 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -2
  FEDCODEC_LIB=$v C=1024 ITERS=3 timeout -k 10 150 python3 tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -1
done; done
