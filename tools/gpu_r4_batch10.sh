#!/bin/bash
# round-4 GPU batch 10: headline encoder WRITE_SIZE, code-word stores ablated (FC_ABL=2) vs the build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/wabl4
mkdir -p $O
for v in "" _abl2; do
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w$v -o run -- python3 bench.py --workload headline --no-cpu-baseline --steps 1 --warmup 1 > $O/w$v.log 2>&1 || exit 1
  python3 - $O/w$v $v <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
  for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
for k, v in acc.items():
  if "encode" in k: print("lib%s %-60s WRITE_SIZE per launch %.4f GB (%d)" % (sys.argv[2], k, sum(v) / len(v) * 1024 / 1e9, len(v)))
PY
done
echo BATCH10_DONE
