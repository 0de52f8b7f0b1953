# A/B of k_encode2 variants: full GPU suite with the last library, then encode times of all (enc_ablate).
# usage: LIBS="federated_amd/libfedcodec_base.so federated_amd/libfedcodec_chain.so" bash tools/diag/ab_chain.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B=${LIBS##* }
FEDCODEC_LIB=$B timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
LIBS="$LIBS $LIBS" CAP=${CAP:-0.6} REPS=5 timeout -k 10 500 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/ab_enc.log || exit 1
cat gpurun_out/ab_enc.log
