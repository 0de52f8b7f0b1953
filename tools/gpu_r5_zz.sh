#!/bin/bash
# round-5 ZZ (final build: rebuild unroll + carried emit checkpoint scan): full GPU suite, smoke, the bench line, then rocprofv3 records of
# the workloads this round's last changes touched
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof8
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5zz_tests.txt 2>&1 || { tail -30 gpurun_out/r5zz_tests.txt; exit 1; }
tail -1 gpurun_out/r5zz_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5zz_smoke.txt 2>&1 || { tail -20 gpurun_out/r5zz_smoke.txt; exit 1; }
tail -1 gpurun_out/r5zz_smoke.txt
timeout -k 10 900 python3 bench.py > gpurun_out/r5zz_bench.json 2> gpurun_out/r5zz_bench.err || { tail -20 gpurun_out/r5zz_bench.err; exit 1; }
head -c 300 gpurun_out/r5zz_bench.json; echo
timeout -k 10 1000 bash tools/profile_workloads.sh gpurun_out/prof8 bare_decode headline_uniform config3 config4_full config4_share headline_c128 > gpurun_out/r5zz_prof.log 2>&1 || { tail -5 gpurun_out/r5zz_prof.log; exit 1; }
tail -1 gpurun_out/r5zz_prof.log
