#!/bin/bash
# round-4 GPU batch 13: checkpointed index emit -- bare-decode tests, then the rebuild timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/diag/idx_ck_debug.py > gpurun_out/ck_debug.txt 2>&1 || exit 5
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_bare_decode.py tests/test_gpu_aggregators.py > gpurun_out/ck_tests.log 2>&1 || { tail -40 gpurun_out/ck_tests.log; exit 1; }
tail -1 gpurun_out/ck_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/idxck -o run -- python3 tools/index_bench.py > gpurun_out/idxck.log 2>&1 || { tail -20 gpurun_out/idxck.log; exit 2; }
rm -f gpurun_out/idxck/*kernel_trace.csv
grep -v "^W2026\|^E2026\|amdgpu.ids" gpurun_out/idxck.log
grep -h "k_idx" gpurun_out/idxck/*kernel_stats.csv | cut -d, -f1-4
