set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gen
timeout -k 10 300 python -u -m pytest tests/test_gpu_quarters.py tests/test_gpu_configs.py tests/test_gpu_codec.py tests/test_gpu_edge_cases.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gen/tests.txt 2>&1 || exit 1
for rep in 1 2; do for L in federated_amd/libfedcodec_gen0.so federated_amd/libfedcodec.so; do
  echo "== $L" >> gpurun_out/gen/ab.txt
  C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=4 FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep decode | tail -2 >> gpurun_out/gen/ab.txt || exit 1
  FEDCODEC_LIB=$L timeout -k 10 200 python bench.py --workload config2 > gpurun_out/gen/b2_$rep_$(basename $L).json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/gen/b2_$rep_$(basename $L).json').read().strip().splitlines()[-1]);print('config2 step', d.get('ms_per_step'), d.get('kernels', ''))" >> gpurun_out/gen/ab.txt
done; done
cat gpurun_out/gen/ab.txt
