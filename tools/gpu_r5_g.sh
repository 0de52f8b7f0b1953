#!/bin/bash
# round-5 G: the full GPU suite (hand-written DFT rotation included), the smoke, the
# default bench line (headline + every single-GPU workload + CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r5g_gputest.txt 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5g_smoke.txt 2>&1 || exit 2
timeout -k 10 600 python3 bench.py > gpurun_out/r5g_bench_line.json 2> gpurun_out/r5g_bench.err || exit 3
