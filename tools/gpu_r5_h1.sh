#!/bin/bash
# round-5 H1: rocprofv3 kernel-trace summaries + FETCH / WRITE passes of the headline,
# headline_uniform, bare_decode and onebit_c128 workloads
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 1100 bash tools/profile_workloads.sh gpurun_out/prof5 headline headline_uniform bare_decode onebit_c128 > gpurun_out/r5h1.log 2>&1 || exit 1
