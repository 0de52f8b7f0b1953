#!/bin/bash
# round-5 SEG: the 8-GPU share (128 x 25 M) by segments per client: FEDCODEC_SEGMENTS 1 (the super-tile encoder
# on whole rows, FEDCODEC_ENC2=1), 2, 4, 8 (default), 16; bench.py headline_c128, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5seg.txt
: > $O
for rep in 1 2; do
  for K in 1 2 4 8 16; do
    E="FEDCODEC_SEGMENTS=$K"
    [ $K = 1 ] && E="$E FEDCODEC_ENC2=1"
    env $E timeout -k 10 300 python3 bench.py --workload headline_c128 --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null > gpurun_out/r5seg_line.json || exit 1
    python3 - "$K" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5seg_line.json"))
v = v["workloads"]["headline_c128"] if "workloads" in v else v
print("segments", sys.argv[1], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "dec", v["decode"]["launch_ms"])
PY
  done
done
cat $O
