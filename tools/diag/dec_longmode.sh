# decoder long-code mode A/B (diagnostic): config 2's shape (8-bit steps) and the headline shape
set -o pipefail
for L in libfedcodec_nolm libfedcodec libfedcodec_nolm libfedcodec; do
  echo "== $L"
  FEDCODEC_LIB=$PWD/federated_amd/$L.so C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=5 timeout -k 10 120 python tools/dec_bench.py 2>&1 | grep decode | tail -2 || exit 1
  FEDCODEC_LIB=$PWD/federated_amd/$L.so C=1024 ITERS=3 timeout -k 10 200 python tools/dec_bench.py 2>&1 | grep decode | tail -2 || exit 1
done
