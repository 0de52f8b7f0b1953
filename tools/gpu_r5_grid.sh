#!/bin/bash
# round-5 GRID: the decoder's persistent grid at the 8-GPU share (128 x 25 M) and the headline: FEDCODEC_DEC_GRID
# 1024 / 1280 (default: 5 workgroups per CU) / 1536 / 2048, bench.py headline_c128, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5grid.txt
: > $O
for rep in 1 2; do
  for G in 1024 1280 1536 2048 3072; do
    FEDCODEC_DEC_GRID=$G timeout -k 10 300 python3 bench.py --workload headline_c128 --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > gpurun_out/r5grid_line.json || exit 1
    python3 - "$G" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5grid_line.json"))
v = v["workloads"]["headline_c128"] if "workloads" in v else v
print("grid", sys.argv[1], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "dec", v["decode"]["launch_ms"])
PY
  done
done
cat $O
