#!/bin/bash
# round-5 A: bare-decode parity (chunk-boundary ends), headline bench line, encoder floor
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bare_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5a_bare.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload headline --no-cpu-baseline > gpurun_out/r5a_head.json 2> gpurun_out/r5a_head.err || exit 2
timeout -k 10 300 python3 tools/floor_bench.py > gpurun_out/r5a_floor.txt 2>&1 || exit 3
