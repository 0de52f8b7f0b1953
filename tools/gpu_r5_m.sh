#!/bin/bash
# round-5 M: full GPU suite, smoke and the bench line on the current build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5m_tests.txt 2>&1 || { tail -30 gpurun_out/r5m_tests.txt; exit 1; }
tail -2 gpurun_out/r5m_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5m_smoke.txt 2>&1 || { tail -20 gpurun_out/r5m_smoke.txt; exit 1; }
tail -2 gpurun_out/r5m_smoke.txt
timeout -k 10 900 python3 bench.py > gpurun_out/r5m_bench.json 2> gpurun_out/r5m_bench.err || { tail -20 gpurun_out/r5m_bench.err; exit 1; }
head -c 400 gpurun_out/r5m_bench.json
