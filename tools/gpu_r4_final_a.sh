#!/bin/bash
# round-4 evidence A: the full GPU suite, the smoke, and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4_gputest_full.txt 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.txt 2>&1 || exit 2
timeout -k 10 500 python3 bench.py > gpurun_out/r4_bench_line.json 2> gpurun_out/r4_bench.err || exit 3
