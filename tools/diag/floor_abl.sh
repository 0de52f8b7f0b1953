# What sets k_encode's uniform floor: ablation builds (FC_ABL bits: 128 no code construction,
# 2 no code stores, 4 no look-back, 1024 no stores and no window clears, 64 synthetic values, no loads)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in base abl128 abl130 abl134 abl1156 abl192; do
  for m in 0 1; do
    FEDCODEC_ENC2=0 FEDCODEC_LIB=federated_amd/libfedcodec_$v.so C=1024 MODE=$m DEC=0 REPS=3 timeout -k 10 150 python -u tools/enc_bench.py 2>&1 | grep -v 'amdgpu.ids\|row bases' >> gpurun_out/floor.log || exit 1
  done
done
cat gpurun_out/floor.log
