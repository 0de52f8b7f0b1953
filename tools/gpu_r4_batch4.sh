#!/bin/bash
# round-4 GPU batch 4: bare-decode parity + index rebuild timing, halves with a small side-decode grid
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bare_decode.py tests/test_gpu_large_p.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_bare3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_idx4 -o idx -- python3 tools/index_bench.py > gpurun_out/index_bench4.txt 2>&1 || exit 2
timeout -k 10 300 python3 tools/overlap_halves.py > gpurun_out/overlap_halves2.txt 2>&1 || exit 3
