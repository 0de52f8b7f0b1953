# k_encode ablations (FC_ABL 4: no look-back, 2: no stream stores) at 128 and 1024 clients (diagnostic)
set -o pipefail
for C in 128 1024; do
  for L in libfedcodec libfedcodec_abl4 libfedcodec_abl2; do
    FEDCODEC_ENC2=0 FEDCODEC_LIB=$PWD/federated_amd/$L.so C=$C MODE=1 DEC=0 REPS=3 timeout -k 10 200 python tools/enc_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  done
done
