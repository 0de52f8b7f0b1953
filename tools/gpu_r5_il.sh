#!/bin/bash
# round-5 IL: the index parse on its own table (L and 4 x runs, one AND per step; default) against the decoder's table (il0):
# bare-string parity tests on the default, then bench.py bare_decode, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bare_decode.py tests/test_gpu_large_p.py > gpurun_out/r5il_tests.txt 2>&1 || { tail -30 gpurun_out/r5il_tests.txt; exit 1; }
tail -1 gpurun_out/r5il_tests.txt
O=gpurun_out/r5il.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec_il0.so federated_amd/libfedcodec.so; do
    FEDCODEC_LIB=$L timeout -k 10 300 python3 bench.py --workload bare_decode --no-cpu-baseline --steps 3 --warmup 1 --extra-steps 5 2>/dev/null > gpurun_out/r5il_line.json || exit 1
    python3 - "$L" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5il_line.json"))
v = v["workloads"]["bare_decode"] if "workloads" in v else v
print(sys.argv[1].split("/")[-1], "step", v["ms_per_step"], "rebuild", v["index_rebuild"]["launch_ms"], "decode", v["decode"]["launch_ms"])
PY
  done
done
cat $O
