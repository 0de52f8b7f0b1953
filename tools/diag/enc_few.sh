# few clients per GPU: super-tile k_encode2 forced on the unsegmented batch vs the default choice
# (one-tile k_encode, or segments).  C values from $CS (default "256 128").
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=federated_amd/libfedcodec.so
: > gpurun_out/enc_few.log
for C in ${CS:-256 128}; do
  C=$C LIBS=$L CAP=0.6 REPS=5 timeout -k 10 300 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc_few.log || exit 1
  SEGMENTS=1 FEDCODEC_ENC2=1 C=$C LIBS=$L CAP=0.6 REPS=5 timeout -k 10 300 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc_few.log || exit 1
  SEGMENTS=1 C=$C LIBS=$L CAP=0.6 REPS=5 timeout -k 10 300 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/enc_few.log || exit 1
done
cat gpurun_out/enc_few.log
