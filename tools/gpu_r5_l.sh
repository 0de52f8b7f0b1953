#!/bin/bash
# round-5 L: cache policy of k_encode2's staging loads (nt) and code stores (nt), and the window ORs as inline asm (no vmcnt wait), A/B, 1024 x 25 M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
L="federated_amd/libfedcodec_base.so federated_amd/libfedcodec_snt.so federated_amd/libfedcodec_cnt.so federated_amd/libfedcodec_bnt.so federated_amd/libfedcodec_easm.so federated_amd/libfedcodec_nnz.so federated_amd/libfedcodec_nnzasm.so"
LIBS="$L $L" CAP=0.5 REPS=5 timeout -k 10 500 python3 -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r5l.txt || exit 1
cat gpurun_out/r5l.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_supertile.py tests/test_gpu_chain.py tests/test_gpu_codec.py > gpurun_out/r5l_tests.txt 2>&1 || { tail -30 gpurun_out/r5l_tests.txt; exit 1; }
tail -2 gpurun_out/r5l_tests.txt
