# k_encode vs k_encode2 (FEDCODEC_ENC2=0/1) across client counts (diagnostic)
set -o pipefail
for C in 128 256 512 1024; do
  for E in 0 1; do
    FEDCODEC_ENC2=$E C=$C MODE=1 DEC=0 REPS=3 timeout -k 10 200 python tools/enc_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 | sed "s/^/enc2=$E /" || exit 1
  done
done
