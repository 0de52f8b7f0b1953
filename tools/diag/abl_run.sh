set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L="federated_amd/libfedcodec_base.so federated_amd/libfedcodec_addc.so federated_amd/libfedcodec_abl8192.so"
LIBS="$L $L" CAP=0.6 REPS=5 timeout -k 10 400 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/abl1.log
