# decoder A/B (tools/dec_bench.py) at several code densities: sparse (trainer-like), config 3, headline
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do for L in $LIBS; do
  for cfg in "C=1024 P=25000000 STEP=0.5 SIGMA=0.15" "C=256 P=4050748 STEP=1.0 SIGMA=1.0" "C=1024 P=25000000 STEP=0.5 SIGMA=0.5" "C=1024 P=25000000 STEP=0.5 SIGMA=1.0"; do
    echo "== $L $cfg" >> gpurun_out/dec_ab2.log
    env $cfg ITERS=4 FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 >> gpurun_out/dec_ab2.log || exit 1
  done
done; done
cat gpurun_out/dec_ab2.log
