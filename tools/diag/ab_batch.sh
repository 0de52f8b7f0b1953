# batch A/B: GPU suite for each variant in $VARS, then encode (enc_ablate) and decode (dec_bench) times
# usage: BASE=federated_amd/libfedcodec_base.so VARS="a.so b.so" bash tools/diag/ab_batch.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/ab_batch.log
for L in $VARS; do
  FEDCODEC_LIB=$L timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests_$(basename $L .so).log 2>&1 || { tail -30 gpurun_out/ab_tests_$(basename $L .so).log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/ab_tests_$(basename $L .so).log)" >> gpurun_out/ab_batch.log
done
LIBS="$BASE $VARS $BASE $VARS" CAP=0.6 REPS=5 timeout -k 10 500 python -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/ab_batch.log || exit 1
for rep in 1 2; do for L in $BASE $VARS; do
  for cfg in "C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25" "C=1024 P=25000000 STEP=0.5 SIGMA=1.0"; do
    echo "== $(basename $L) $cfg" >> gpurun_out/ab_batch.log
    env $cfg ITERS=4 FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 >> gpurun_out/ab_batch.log || exit 1
  done
done; done
cat gpurun_out/ab_batch.log
