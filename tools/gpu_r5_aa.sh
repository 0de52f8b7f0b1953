#!/bin/bash
# round-5 AA: k_decode lane segments for the 8-GPU share (128 x 25 M): span 1 / 2 tiles and
# 64 / 128 lanes per tile (FEDCODEC_DEC_SPAN, FEDCODEC_DEC_LPT), bench.py headline_c128, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5aa.txt
: > $O
for rep in 1 2; do
  for cfg in "1 128" "1 64" "2 128" "2 64"; do
    set -- $cfg
    FEDCODEC_DEC_SPAN=$1 FEDCODEC_DEC_LPT=$2 timeout -k 10 300 python3 bench.py --workload headline_c128 --no-cpu-baseline --steps 3 --warmup 1 --extra-steps 10 2>/dev/null > gpurun_out/r5aa_line.json || exit 1
    python3 - "$1" "$2" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5aa_line.json"))
v = v["workloads"]["headline_c128"] if "workloads" in v else v
print("span", sys.argv[1], "lpt", sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "dec", v["decode"]["launch_ms"])
PY
  done
done
cat $O
