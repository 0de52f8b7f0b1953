#!/bin/bash
# round-5 P: non-temporal row reads in k_mask_encode / k_client_norms (FC_ROW_NT=1, rnt)
# against the default build: bench.py's onebit, onebit_c128 and trainer_round lines, twice
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5p.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec.so federated_amd/libfedcodec_rnt.so; do
    for w in onebit onebit_c128 trainer_round; do
      FEDCODEC_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 3 --warmup 1 --extra-steps 5 2>/dev/null > gpurun_out/r5p_line.json || exit 1
      python3 - "$L" "$w" >> $O <<'PY'
import json, sys
d = json.load(open("gpurun_out/r5p_line.json"))
v = d["workloads"][sys.argv[2]] if "workloads" in d else d
print(sys.argv[1].split("/")[-1], sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], v["roofline"]["frac"],
      "norms", (v.get("norms_roofline") or {}).get("launch_ms"), (v.get("norms_roofline") or {}).get("frac"))
PY
    done
  done
done
cat $O
