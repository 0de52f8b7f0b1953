#!/bin/bash
# round-5 REGR: the headline encoder on the final build against the build of the round's final bench line
# (prev = commit 9634c20): is the look-back safety net (cold code inlined into k_encode2) free? bench.py
# headline / headline_uniform, alternating, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5regr.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec_prev.so federated_amd/libfedcodec.so; do
    for w in headline headline_uniform; do
      FEDCODEC_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null > gpurun_out/r5regr_line.json || exit 1
      python3 - "$L" "$w" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5regr_line.json"))
v = v["workloads"][sys.argv[2]] if "workloads" in v and sys.argv[2] in v["workloads"] else v
print(sys.argv[1].split("/")[-1], sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "frac", v["roofline"]["frac"])
PY
    done
  done
done
cat $O
