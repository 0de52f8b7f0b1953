#!/bin/bash
# round-4 evidence C: full GPU suite + smoke + bench line (evidence A), aux_bench, index rebuild split
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/gpu_r4_final_a.sh || exit $?
tail -1 gpurun_out/r4_gputest_full.txt
timeout -k 10 300 python3 tools/aux_bench.py > gpurun_out/aux_bench_r4b.txt 2>&1 || exit 5
cat gpurun_out/aux_bench_r4b.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/idxsplit5 -o run -- python3 tools/index_bench.py headline > gpurun_out/idxsplit5.log 2>&1 || exit 6
rm -f gpurun_out/idxsplit5/*kernel_trace.csv
grep -v "^W2026\|^E2026\|amdgpu.ids" gpurun_out/idxsplit5.log
grep -h "k_idx" gpurun_out/idxsplit5/*kernel_stats.csv | cut -d, -f1-4
