#!/bin/bash
# round-4 GPU batch 15: full suite + smoke + bench on the current build, then the index rebuild's kernel split
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_r4_final_a.sh || exit $?
tail -1 gpurun_out/r4_gputest_full.txt
for w in headline config2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/idxsplit2_$w -o run -- python3 tools/index_bench.py $w > gpurun_out/idxsplit2_$w.log 2>&1 || exit 4
  rm -f gpurun_out/idxsplit2_$w/*kernel_trace.csv
  grep -v "^W2026\|^E2026\|amdgpu.ids" gpurun_out/idxsplit2_$w.log
  grep -h "k_idx" gpurun_out/idxsplit2_$w/*kernel_stats.csv | cut -d, -f1-4
done
