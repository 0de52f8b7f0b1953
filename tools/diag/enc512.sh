# 512 clients x 25 M (one GPU's share at N = 2): one-tile k_encode vs super-tile k_encode2 vs two segments
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=federated_amd/libfedcodec.so
: > gpurun_out/enc512.log
C=512 LIBS=$L CAP=0.6 REPS=5 timeout -k 10 300 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc512.log || exit 1
FEDCODEC_ENC2=1 C=512 LIBS=$L CAP=0.6 REPS=5 timeout -k 10 300 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc512.log || exit 1
SEGMENTS=2 C=512 LIBS=$L CAP=0.6 REPS=5 timeout -k 10 300 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc512.log || exit 1
cat gpurun_out/enc512.log
