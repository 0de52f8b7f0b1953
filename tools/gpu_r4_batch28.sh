#!/bin/bash
# round-4 GPU batch 28: the guessed parse's wave-uniform fast steps (default) vs FC_IDX_UNIFORM=0
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_bare_decode.py tests/test_gpu_aggregators.py tests/test_gpu_large_p.py > gpurun_out/b28_tests.log 2>&1 || { tail -40 gpurun_out/b28_tests.log; exit 1; }
tail -1 gpurun_out/b28_tests.log
for rep in 1 2; do for v in "" _nouni; do
  echo "== lib$v"
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so timeout -k 10 200 python3 tools/index_bench.py 2>&1 | grep -v amdgpu.ids || exit 2
done; done
