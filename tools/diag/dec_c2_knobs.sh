# config-2 decoder: launch knobs (lanes per unit, grid) on the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/dec_c2_knobs.log
for rep in 1 2; do for kn in "X=0" "FEDCODEC_DEC_LPT=64" "FEDCODEC_DEC_LPT=256" "FEDCODEC_DEC_GRID=1024" "FEDCODEC_DEC_GRID=4096"; do
  echo "== $kn" >> gpurun_out/dec_c2_knobs.log
  env $kn C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=5 timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep decode | tail -2 >> gpurun_out/dec_c2_knobs.log || exit 1
done; done
cat gpurun_out/dec_c2_knobs.log
