#!/bin/bash
# round-5 WPE6: the decoder held to 80 VGPRs (FC_DEC_WPE=6, 17 spilled) at 6 workgroups per CU (grid 1536) against the
# default (96 VGPRs, 5 per CU): does more latency hiding pay for the spills? decoder parity on wpe6, then bench.py
# headline / headline_c128, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
FEDCODEC_LIB=federated_amd/libfedcodec_wpe6.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_codec.py > gpurun_out/r5w6_tests.txt 2>&1 || { tail -30 gpurun_out/r5w6_tests.txt; exit 1; }
tail -1 gpurun_out/r5w6_tests.txt
O=gpurun_out/r5w6.txt
: > $O
for rep in 1 2; do
  for V in "federated_amd/libfedcodec.so 0" "federated_amd/libfedcodec_wpe6.so 1536" "federated_amd/libfedcodec_wpe6.so 1280"; do
    set -- $V
    for w in headline headline_c128; do
      E=""; [ "$2" != 0 ] && E="FEDCODEC_DEC_GRID=$2"
      env FEDCODEC_LIB=$1 $E timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null > gpurun_out/r5w6_line.json || exit 1
      python3 - "$1" "$2" "$w" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5w6_line.json"))
v = v["workloads"][sys.argv[3]] if "workloads" in v and sys.argv[3] in v["workloads"] else v
print(sys.argv[1].split("/")[-1], "grid", sys.argv[2], sys.argv[3], "step", v["ms_per_step"], "dec", v["decode"]["launch_ms"])
PY
    done
  done
done
cat $O
