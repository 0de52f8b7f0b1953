# one-bit codec A/B of library variants (tools/onebit_bench.py), interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in ${REPS_AB:-1 2}; do for L in $LIBS; do
  echo "== $L" >> gpurun_out/ob_ab.log
  FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/onebit_bench.py 2>&1 | grep -v amdgpu.ids >> gpurun_out/ob_ab.log || exit 1
done; done
cat gpurun_out/ob_ab.log
