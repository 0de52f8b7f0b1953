# k_encode at a fixed 3.2 G elements split over 128..1024 clients (diagnostic: per-client vs per-element cost)
set -o pipefail
for CP in 128:25000000 256:12500000 512:6250000 1024:3125000 128:50000000; do
  C=${CP%%:*}; P=${CP##*:}
  FEDCODEC_ENC2=0 C=$C P=$P MODE=1 DEC=0 REPS=3 timeout -k 10 200 python tools/enc_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
done
