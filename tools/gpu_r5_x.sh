#!/bin/bash
# round-5 X: client-split grids 1x / 2x / 4x the resident workgroups (FEDCODEC_PARTS_MULT):
# one-bit (1024 and 128 clients) and the trainer round's client norms, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5x.txt
: > $O
for rep in 1 2; do
  for m in 1 2 4; do
    for w in onebit onebit_c128 trainer_round trainer_round_c128; do
      FEDCODEC_PARTS_MULT=$m timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 3 --warmup 1 --extra-steps 5 2>/dev/null > gpurun_out/r5x_line.json || exit 1
      python3 - "$m" "$w" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5x_line.json"))
v = v["workloads"][sys.argv[2]] if "workloads" in v else v
n = v.get("norms_roofline") or {}
print("mult", sys.argv[1], sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], v["roofline"]["frac"], "norms", n.get("launch_ms"), n.get("frac"))
PY
    done
  done
done
cat $O
