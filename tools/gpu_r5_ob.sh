#!/bin/bash
# round-5 OB: the one-bit mask encoder: float32 tile partials for the sums of x (f32x), one tile per wave at a time (np), both (f32xnp), against the default (base):
# (base): bench.py onebit_c128 and onebit, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5ob.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec.so federated_amd/libfedcodec_f32x.so federated_amd/libfedcodec_np.so federated_amd/libfedcodec_f32xnp.so; do
    for w in onebit_c128 onebit; do
      FEDCODEC_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null > gpurun_out/r5ob_line.json || exit 1
      python3 - "$L" "$w" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5ob_line.json"))
v = v["workloads"][sys.argv[2]] if "workloads" in v else v
print(sys.argv[1].split("/")[-1], sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "frac", v["roofline"]["frac"])
PY
    done
  done
done
cat $O
