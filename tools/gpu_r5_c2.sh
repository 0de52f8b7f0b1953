#!/bin/bash
# round-5 config 2 experiment: the one-tile encoder + quarter index (default) against the
# plain tile index, and the super-tile encoder (FEDCODEC_ENC2=1, NT=2) with the plain index
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/c2
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --workload config2 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/c2/$tag.json 2> gpurun_out/c2/$tag.err || { tail -5 gpurun_out/c2/$tag.err; return 1; }
  env "$@" timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2/$tag -o run -- python3 bench.py --workload config2 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/c2/$tag.log 2>&1 || { tail -5 gpurun_out/c2/$tag.log; return 1; }
  find gpurun_out/c2/$tag -name "*kernel_trace.csv" -delete
  python3 - gpurun_out/c2/$tag $tag <<'PY'
import csv, glob, json, sys
d, tag = sys.argv[1], sys.argv[2]
line = json.loads(open(d + ".json").read().strip().splitlines()[-1])
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
ks = {r["Name"]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f)) if "::k_" in r["Name"]}
top = sorted(ks.items(), key=lambda kv: -kv[1])[:4]
print(tag, "ms_per_step %.4f" % line["ms_per_step"], " ".join("%s=%.1fus" % (k.split("::")[1].split("(")[0][:40], v) for k, v in top))
PY
}
run base FEDCODEC_X=0 && run noq FEDCODEC_QUARTERS=0 && run enc2 FEDCODEC_QUARTERS=0 FEDCODEC_ENC2=1 && run enc2q4 FEDCODEC_QUARTERS=0 FEDCODEC_ENC2=1 FEDCODEC_ENC_NT=4
