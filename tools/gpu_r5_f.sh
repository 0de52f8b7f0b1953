#!/bin/bash
# round-5 F (final build: look-back timeout flag-only, index-parse table, decoder span knob, mask-encoder knobs): full GPU suite, smoke, the bench line, then rocprofv3 records
# the workloads this round's last changes touched
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof10
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r5f_tests.txt 2>&1 || { tail -30 gpurun_out/r5f_tests.txt; exit 1; }
tail -1 gpurun_out/r5f_tests.txt
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5f_smoke.txt 2>&1 || { tail -20 gpurun_out/r5f_smoke.txt; exit 1; }
tail -1 gpurun_out/r5f_smoke.txt
timeout -k 10 900 python3 bench.py > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || { tail -20 gpurun_out/r5f_bench.err; exit 1; }
head -c 300 gpurun_out/r5f_bench.json; echo
timeout -k 10 1000 bash tools/profile_workloads.sh gpurun_out/prof10 bare_decode headline > gpurun_out/r5f_prof.log 2>&1 || { tail -5 gpurun_out/r5f_prof.log; exit 1; }
tail -1 gpurun_out/r5f_prof.log
