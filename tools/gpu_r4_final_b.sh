#!/bin/bash
# round-4 evidence B: rocprofv3 kernel stats + separate FETCH_SIZE / WRITE_SIZE passes per workload
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/profile_workloads.sh gpurun_out/prof_r4 ${WL:-headline headline_uniform trainer_round} > gpurun_out/prof_r4_b.log 2>&1
