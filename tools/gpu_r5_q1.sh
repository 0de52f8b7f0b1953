#!/bin/bash
# round-5 Q1: the bench line on the current build, then rocprofv3 kernel-trace summaries and
# FETCH / WRITE passes of six workloads (profiles/r05 records)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof6
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_supertile.py -k edge > gpurun_out/r5q_tests.txt 2>&1 || { tail -30 gpurun_out/r5q_tests.txt; exit 1; }
tail -1 gpurun_out/r5q_tests.txt
timeout -k 10 900 python3 bench.py > gpurun_out/r5q_bench.json 2> gpurun_out/r5q_bench.err || { tail -20 gpurun_out/r5q_bench.err; exit 1; }
head -c 300 gpurun_out/r5q_bench.json; echo
timeout -k 10 1000 bash tools/profile_workloads.sh gpurun_out/prof6 headline headline_uniform trainer_round onebit onebit_c128 headline_c128 > gpurun_out/r5q1.log 2>&1 || { tail -5 gpurun_out/r5q1.log; exit 1; }
tail -2 gpurun_out/r5q1.log
