# config-2 decoder A/B of library variants: LIBS="a.so b.so" bash tools/diag/dec_ab_c2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/dec_ab_c2.log
for rep in 1 2; do for L in $LIBS; do
  echo "== $L" >> gpurun_out/dec_ab_c2.log
  C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=5 FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep decode | tail -2 >> gpurun_out/dec_ab_c2.log || exit 1
done; done
cat gpurun_out/dec_ab_c2.log
