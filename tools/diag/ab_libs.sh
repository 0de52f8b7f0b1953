# A/B of library variants: parity suite with B, then encode/decode times of A and B interleaved.
# usage: A=federated_amd/libfedcodec_base.so B=federated_amd/libfedcodec_x.so bash tools/diag/ab_libs.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FEDCODEC_LIB=$B timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for rep in 1 2; do
  for L in $A $B; do
    for cfg in "C=1024 MODE=1" "C=1024 MODE=0" "C=128 MODE=1" ${EXTRA_CFG}; do
      env $cfg FEDCODEC_LIB=$L REPS=5 timeout -k 10 150 python -u tools/enc_bench.py 2>&1 | grep -v 'amdgpu.ids\|row bases' >> gpurun_out/ab.log || exit 1
    done
  done
done
cat gpurun_out/ab.log
