#!/bin/bash
# round-4 GPU batch 31: the default build with the one-refill LONG loop -- full GPU suite, smoke, default bench line,
# rocprofv3 records of config 2 (kernel stats + FETCH / WRITE passes)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r4_gputest_full.txt 2>&1 || { tail -30 gpurun_out/r4_gputest_full.txt; exit 1; }
tail -1 gpurun_out/r4_gputest_full.txt
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.txt 2>&1 || exit 2
timeout -k 10 500 python3 bench.py > gpurun_out/r4_bench_line.json 2> gpurun_out/r4_bench.err || exit 3
head -c 300 gpurun_out/r4_bench_line.json; echo
rm -rf gpurun_out/prof_r4c2
bash tools/profile_workloads.sh gpurun_out/prof_r4c2 config2 > gpurun_out/prof_r4c2.log 2>&1 || exit 4
