#!/bin/bash
# round-4 GPU batch 29: the checkpointed emit (k_idx_emit) at 4 (default) / 5 / 6 waves per SIMD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in _emit5 _emit6; do
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_bare_decode.py > gpurun_out/b29_tests$v.log 2>&1 || { tail -40 gpurun_out/b29_tests$v.log; exit 1; }
  tail -1 gpurun_out/b29_tests$v.log
done
for rep in 1 2; do for v in "" _emit5 _emit6; do
  echo "== lib$v"
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so timeout -k 10 200 python3 tools/index_bench.py 2>&1 | grep -v amdgpu.ids || exit 2
done; done
