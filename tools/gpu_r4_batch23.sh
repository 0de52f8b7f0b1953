#!/bin/bash
# round-4 GPU batch 23: index rebuild chunk size / checkpoint count variants -- bare-decode tests + timing each
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in ix8192_15 ix2048_3 ix4096_15; do
  L=$PWD/federated_amd/libfedcodec_$v.so
  echo "== $v"
  FEDCODEC_LIB=$L timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_bare_decode.py > gpurun_out/b23_$v.log 2>&1 || { tail -30 gpurun_out/b23_$v.log; exit 1; }
  tail -1 gpurun_out/b23_$v.log
  FEDCODEC_LIB=$L timeout -k 10 200 python3 tools/index_bench.py 2>&1 | grep -v amdgpu.ids || exit 2
done
echo "== default"
timeout -k 10 200 python3 tools/index_bench.py 2>&1 | grep -v amdgpu.ids || exit 3
