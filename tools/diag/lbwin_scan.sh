# k_encode look-back prefetch window at few clients per GPU (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT
for C in ${CS:-128 256}; do for w in ${WINS:-12 16 20 24 32 40 48 64}; do
  echo "C=$C lbwin=$w" >> gpurun_out/lbwin.log
  FEDCODEC_LB_WIN=$w C=$C DEC=0 REPS=7 FEDCODEC_ENC2=0 timeout -k 10 100 python -u tools/enc_bench.py 2>&1 | grep -v 'amdgpu.ids\|row bases' >> gpurun_out/lbwin.log || exit 1
done; done
cat gpurun_out/lbwin.log
