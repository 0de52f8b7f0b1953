# decoder A/B on config 2 (8-bit steps, 128 clients) and the headline density:
# LIBS="a.so b.so" bash tools/diag/ab_dec2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/dec_ab2.log
for rep in 1 2; do for L in $LIBS; do
  for cfg in "C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25" ${HEADLINE:+"C=1024 P=25000000 STEP=0.5 SIGMA=1.0"}; do
    echo "== $L $cfg $(env $cfg ITERS=6 FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -3 | tr '\n' ' ')" >> gpurun_out/dec_ab2.log || exit 1
  done
done; done
cat gpurun_out/dec_ab2.log
