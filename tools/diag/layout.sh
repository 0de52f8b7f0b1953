set -o pipefail
for L in sep pack skew; do
  for M in 1 0; do
    LAYOUT=$L MODE=$M C=1024 timeout -k 10 150 python -u tools/enc_bench.py >> gpurun_out/layout.log 2>&1 || exit 1
  done
done
for L in sep skew; do
  LAYOUT=$L MODE=1 C=128 timeout -k 10 100 python -u tools/enc_bench.py >> gpurun_out/layout.log 2>&1 || exit 1
done
