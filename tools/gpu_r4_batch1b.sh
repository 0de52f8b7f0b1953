#!/bin/bash
# round-4 GPU batch 1b: the co-scheduling experiments
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/overlap_halves.py > gpurun_out/overlap_halves.txt 2>&1 || exit 5
timeout -k 10 300 python3 tools/overlap_xbatch.py > gpurun_out/overlap_xbatch.txt 2>&1 || exit 4
