#!/bin/bash
# round-5 S: the one-tile k_encode with the same store loop (current) against the previous
# commit (prev): encoder parity tests, then bench.py's config2 / config3 / config4_share /
# headline_c128 lines, two interleaved passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec.py tests/test_gpu_configs.py tests/test_gpu_segmented.py > gpurun_out/r5s_tests.txt 2>&1 || { tail -30 gpurun_out/r5s_tests.txt; exit 1; }
tail -1 gpurun_out/r5s_tests.txt
O=gpurun_out/r5s.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec_prev.so federated_amd/libfedcodec.so; do
    for w in config2 config3 config4_share headline_c128; do
      FEDCODEC_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 3 --warmup 1 --extra-steps 10 2>/dev/null > gpurun_out/r5s_line.json || exit 1
      python3 - "$L" "$w" >> $O <<'PY'
import json, sys
d = json.load(open("gpurun_out/r5s_line.json"))
v = d["workloads"][sys.argv[2]] if "workloads" in d else d
print(sys.argv[1].split("/")[-1], sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], v["roofline"]["frac"], "dec", v["decode"]["launch_ms"])
PY
    done
  done
done
cat $O
