#!/bin/bash
# round-5 SEGNT: the segmented encoder's stitch with non-temporal segment reads and stream stores (segnt) against
# the default: segmented-encode parity tests on segnt, then bench.py headline_c128 / config3 / config4_share, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
FEDCODEC_LIB=federated_amd/libfedcodec_segnt.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_segmented.py > gpurun_out/r5sn_tests.txt 2>&1 || { tail -30 gpurun_out/r5sn_tests.txt; exit 1; }
tail -1 gpurun_out/r5sn_tests.txt
O=gpurun_out/r5sn.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec.so federated_amd/libfedcodec_segnt.so; do
    for w in headline_c128 config3 config4_share; do
      FEDCODEC_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null > gpurun_out/r5sn_line.json || exit 1
      python3 - "$L" "$w" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5sn_line.json"))
v = v["workloads"][sys.argv[2]] if "workloads" in v else v
print(sys.argv[1].split("/")[-1], sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "dec", v["decode"]["launch_ms"])
PY
    done
  done
done
cat $O
