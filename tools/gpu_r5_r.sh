#!/bin/bash
# round-5 R: k_encode2 code stores with the capacity bound hoisted and a ticket-uniform funnel, window zeroed 16 bytes per lane (current) against the previous commit (prev)
# encoder parity tests first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_supertile.py tests/test_gpu_chain.py tests/test_gpu_codec.py > gpurun_out/r5r_tests.txt 2>&1 || { tail -30 gpurun_out/r5r_tests.txt; exit 1; }
tail -1 gpurun_out/r5r_tests.txt
L="federated_amd/libfedcodec_prev.so federated_amd/libfedcodec.so"
LIBS="$L $L $L" CAP=0.5 REPS=5 timeout -k 10 500 python3 -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r5r.txt || exit 1
cat gpurun_out/r5r.txt
