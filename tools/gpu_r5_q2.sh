#!/bin/bash
# round-5 Q2: the same records for six more workloads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof6
timeout -k 10 1100 bash tools/profile_workloads.sh gpurun_out/prof6 config4_full config4_share config3 config2 trainer_round_c128 bare_decode > gpurun_out/r5q2.log 2>&1 || { tail -5 gpurun_out/r5q2.log; exit 1; }
tail -2 gpurun_out/r5q2.log
