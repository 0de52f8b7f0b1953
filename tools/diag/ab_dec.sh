# decoder A/B of library variants: LIBS="a.so b.so" bash tools/diag/ab_dec.sh
# (tools/dec_bench.py: config 2 (8-bit steps), config 3, headline density at 1024 clients)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/dec_ab.log
for rep in 1 2; do for L in $LIBS; do
  for cfg in "C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25" "C=256 P=4050748 STEP=1.0 SIGMA=1.0" "C=1024 P=25000000 STEP=0.5 SIGMA=1.0"; do
    echo "== $L $cfg" >> gpurun_out/dec_ab.log
    env $cfg ITERS=4 FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/dec_ab.log || exit 1
  done
done; done
cat gpurun_out/dec_ab.log
