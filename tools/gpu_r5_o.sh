#!/bin/bash
# round-5 O: k_encode2's distortion on the matrix pipe (FC_DIST_MFMA=1) -- encoder parity
# tests through that build, then its encode time against the default build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
FEDCODEC_LIB=federated_amd/libfedcodec_mfma.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_supertile.py tests/test_gpu_chain.py tests/test_gpu_codec.py tests/test_gpu_aggregators.py > gpurun_out/r5o_tests.txt 2>&1 || { tail -30 gpurun_out/r5o_tests.txt; exit 1; }
tail -1 gpurun_out/r5o_tests.txt
L="federated_amd/libfedcodec.so federated_amd/libfedcodec_mfma.so"
LIBS="$L $L $L" CAP=0.5 REPS=5 timeout -k 10 500 python3 -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r5o.txt || exit 1
cat gpurun_out/r5o.txt
