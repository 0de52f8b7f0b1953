#!/bin/bash
# round-4 GPU batch 17: guessed parse with unchecked double steps away from the chunk end -- tests, rebuild split
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_bare_decode.py tests/test_gpu_aggregators.py tests/test_gpu_large_p.py > gpurun_out/b17_tests.log 2>&1 || { tail -40 gpurun_out/b17_tests.log; exit 1; }
tail -1 gpurun_out/b17_tests.log
for w in headline config2 config3; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/idxsplit4_$w -o run -- python3 tools/index_bench.py $w > gpurun_out/idxsplit4_$w.log 2>&1 || exit 4
  rm -f gpurun_out/idxsplit4_$w/*kernel_trace.csv
  grep -v "^W2026\|^E2026\|amdgpu.ids" gpurun_out/idxsplit4_$w.log
  grep -h "k_idx_spec\|k_idx_emit" gpurun_out/idxsplit4_$w/*kernel_stats.csv | cut -d, -f1-4
done
