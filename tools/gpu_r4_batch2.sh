#!/bin/bash
# round-4 GPU batch 2: host-resident rates (both codecs, one GPU's 128-client share), default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/e2e_host.py --clients 128 --batch 16 --codec rlgamma > gpurun_out/e2e_rlgamma_c128.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/e2e_host.py --clients 128 --batch 16 --codec onebit > gpurun_out/e2e_onebit_c128.txt 2>&1 || exit 2
timeout -k 10 500 python3 bench.py > gpurun_out/bench_r4a.json 2> gpurun_out/bench_r4a.err || exit 3
