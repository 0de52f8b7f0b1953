#!/bin/bash
# round-4 GPU batch: new parity tests, encoder floor, bare-code index profile, co-scheduling experiment
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bare_decode.py tests/test_gpu_pipeline.py tests/test_gpu_large_p.py tests/test_gpu_aggregators.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_bare2.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/floor_bench.py > gpurun_out/floor.txt 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_idx3 -o idx -- python3 tools/index_bench.py > gpurun_out/index_bench3.txt 2>&1 || exit 3
timeout -k 10 300 python3 tools/overlap_xbatch.py > gpurun_out/overlap_xbatch.txt 2>&1 || exit 4
timeout -k 10 300 python3 tools/overlap_halves.py > gpurun_out/overlap_halves.txt 2>&1 || exit 5
