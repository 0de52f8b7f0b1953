#!/bin/bash
# round-5 W: one-bit mask encoder at 1024 x 25 M with 1 / 2 / 4 parts per client
# (FEDCODEC_OB_PARTS; the default is 1 there), bench.py's onebit line, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w.txt
: > $O
for rep in 1 2; do
  for np in 1 2 4; do
    FEDCODEC_OB_PARTS=$np timeout -k 10 300 python3 bench.py --workload onebit --no-cpu-baseline --steps 3 --warmup 1 --extra-steps 5 2>/dev/null > gpurun_out/r5w_line.json || exit 1
    python3 - "$np" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5w_line.json"))
v = v["workloads"]["onebit"] if "workloads" in v else v
print("parts", sys.argv[1], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], v["roofline"]["frac"], "dec", v["decode"]["launch_ms"])
PY
  done
done
cat $O
