#!/bin/bash
# round-5 SPAN4: the decoder's parity tests with two- and four-tile lane segments, then bench.py headline
# and bare_decode with FEDCODEC_DEC_SPAN 2 (default) / 4, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_decoder_span.py > gpurun_out/r5s4_tests.txt 2>&1 || { tail -30 gpurun_out/r5s4_tests.txt; exit 1; }
tail -1 gpurun_out/r5s4_tests.txt
O=gpurun_out/r5s4.txt
: > $O
for rep in 1 2; do
  for S in 2 4; do
    FEDCODEC_DEC_SPAN=$S timeout -k 10 300 python3 bench.py --workload headline --no-cpu-baseline --steps 3 --warmup 1 2>/dev/null > gpurun_out/r5s4_line.json || exit 1
    python3 - "$S" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5s4_line.json"))
v = v["workloads"]["headline"] if "workloads" in v and "headline" in v["workloads"] else v
print("span", sys.argv[1], "headline step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "dec", v["decode"]["launch_ms"])
PY
  done
done
cat $O
