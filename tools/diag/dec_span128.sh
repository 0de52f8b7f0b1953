# decoder lane-segment span at few clients per GPU (the 8-GPU share 128 x 25 M, config 4's share 64 x 11 M)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/dec_span.log
for rep in 1 2; do for sp in 1 2; do
  for cfg in "C=128 P=25000000" "C=64 P=11000000"; do
    echo "== span $sp $cfg" >> gpurun_out/dec_span.log
    env $cfg FEDCODEC_DEC_SPAN=$sp ITERS=4 timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/dec_span.log || exit 1
  done
done; done
cat gpurun_out/dec_span.log
