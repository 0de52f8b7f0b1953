#!/bin/bash
# round-5 H2: the same for trainer_round_c128, config4_full, onebit and config2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 1100 bash tools/profile_workloads.sh gpurun_out/prof5 trainer_round_c128 config4_full onebit config2 > gpurun_out/r5h2.log 2>&1 || exit 1
