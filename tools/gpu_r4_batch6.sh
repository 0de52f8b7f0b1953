#!/bin/bash
# round-4 GPU batch 6: XCD-group ticket streams (FEDCODEC_XCD_SHARD=1, default) vs the old
# mapping (=0): encoder-side GPU tests, step times per workload, headline WRITE_SIZE
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/xcd
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_configs.py tests/test_gpu_supertile.py tests/test_gpu_chain.py tests/test_gpu_codec.py \
  tests/test_gpu_segmented.py tests/test_gpu_quarters.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for x in 1 0; do for w in headline headline_uniform config2 config3 headline_c128; do
  FEDCODEC_XCD_SHARD=$x timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 --extra-steps 5 > $O/b_${w}_$x.json 2> $O/b_${w}_$x.err || exit 2
  python3 - $O/b_${w}_$x.json $w $x <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = sys.argv[2]
r = d if w == "headline" else d["workloads"][w]
print("xcd=%s %-18s step %.3f ms  encode %.3f ms" % (sys.argv[3], w, r["ms_per_step"], r["roofline"]["launch_ms"]), flush=True)
PY
done; done; done
for x in 1 0; do
  FEDCODEC_XCD_SHARD=$x timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$x -o run -- python3 bench.py --workload headline --no-cpu-baseline --steps 2 --warmup 1 > $O/write_$x.log 2>&1 || exit 3
  python3 - $O/write_$x $x <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
  for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:50]].append(float(r["Counter_Value"]))
for k, v in acc.items():
  if "encode" in k: print("xcd=%s %-50s WRITE_SIZE per launch %.3f GB" % (sys.argv[2], k, sum(v) / len(v) * 1024 / 1e9))
PY
done
echo BATCH6_DONE
