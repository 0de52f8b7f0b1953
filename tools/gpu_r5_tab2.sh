#!/bin/bash
# round-5 TAB2: the decoder's table steps on byte fields + a separate bits table (FC_DEC_TAB2=1, tab2) against the
# default: decoder parity tests on tab2 (codec, aggregators, span, quarters, bare strings), then bench.py headline /
# headline_c128 / config2 / config3, two passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
FEDCODEC_LIB=federated_amd/libfedcodec_tab2.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_codec.py tests/test_gpu_decoder_span.py tests/test_gpu_quarters.py tests/test_gpu_bare_decode.py > gpurun_out/r5t2_tests.txt 2>&1 || { tail -30 gpurun_out/r5t2_tests.txt; exit 1; }
tail -1 gpurun_out/r5t2_tests.txt
O=gpurun_out/r5t2.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec.so federated_amd/libfedcodec_tab2.so; do
    for w in headline headline_c128 config2 config3; do
      FEDCODEC_LIB=$L timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 2>/dev/null > gpurun_out/r5t2_line.json || exit 1
      python3 - "$L" "$w" >> $O <<'PY'
import json, sys
v = json.load(open("gpurun_out/r5t2_line.json"))
v = v["workloads"][sys.argv[2]] if "workloads" in v and sys.argv[2] in v["workloads"] else v
print(sys.argv[1].split("/")[-1], sys.argv[2], "step", v["ms_per_step"], "enc", v["roofline"]["launch_ms"], "dec", v["decode"]["launch_ms"])
PY
    done
  done
done
cat $O
