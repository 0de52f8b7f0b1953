#!/bin/bash
# round-5 T: k_encode2 micro-steps -- ss = no max-scan when every lane has a nonzero
# (FC_SCAN_SKIP), rm = run code emitted with the first chunk pair (FC_RUN_MERGE), ssrm = both;
# parity tests through ssrm, then encode times against the default build, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
FEDCODEC_LIB=federated_amd/libfedcodec_ssrm.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_supertile.py tests/test_gpu_chain.py tests/test_gpu_codec.py > gpurun_out/r5t_tests.txt 2>&1 || { tail -30 gpurun_out/r5t_tests.txt; exit 1; }
tail -1 gpurun_out/r5t_tests.txt
L="federated_amd/libfedcodec.so federated_amd/libfedcodec_ss.so federated_amd/libfedcodec_rm.so federated_amd/libfedcodec_ssrm.so"
LIBS="$L $L" CAP=0.5 REPS=5 timeout -k 10 500 python3 -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r5t.txt || exit 1
cat gpurun_out/r5t.txt
