# config-2 encoder launch knobs through bench.py --workload config2 (encoder launch ms from the line)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/enc_c2_knobs.log
for rep in 1 2; do for kn in "X=0" "FEDCODEC_ENC_GRID=2048" "FEDCODEC_ENC_GRID=3072" "FEDCODEC_ENC_GRID=6144" "FEDCODEC_LB_WIN=16" "FEDCODEC_LB_WIN=32"; do
  env $kn timeout -k 10 200 python bench.py --workload config2 --no-cpu-baseline > gpurun_out/enc_c2.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/enc_c2.json').read().strip().splitlines()[-1]);w=d.get('workloads',{}).get('config2',d);print('$kn', w['ms_per_step'], w['roofline']['launch_ms'], w['decode']['launch_ms'])" >> gpurun_out/enc_c2_knobs.log
done; done
cat gpurun_out/enc_c2_knobs.log
