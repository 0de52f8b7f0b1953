#!/bin/bash
# round-5 U: k_encode2 per-tile emission without the window clamp (guarded per tile)
# (current) against the previous commit (prev), and the chunks
# quantised before coding (qf, FC_QUANT_FIRST=1); parity tests through qf and current first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for L in federated_amd/libfedcodec_qf.so federated_amd/libfedcodec.so; do
FEDCODEC_LIB=$L timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_supertile.py tests/test_gpu_chain.py tests/test_gpu_codec.py > gpurun_out/r5u_tests.txt 2>&1 || { tail -30 gpurun_out/r5u_tests.txt; exit 1; }
tail -1 gpurun_out/r5u_tests.txt
done
L="federated_amd/libfedcodec_prev.so federated_amd/libfedcodec.so federated_amd/libfedcodec_qf.so"
LIBS="$L $L $L" CAP=0.5 REPS=5 timeout -k 10 500 python3 -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r5u.txt || exit 1
cat gpurun_out/r5u.txt
