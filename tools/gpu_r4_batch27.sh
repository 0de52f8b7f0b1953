#!/bin/bash
# round-4 GPU batch 27: index rebuild kernels' SQ counters at the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/pmc_idx
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $O/p1 -o run -- python3 tools/index_bench.py headline > $O/p1.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS --output-format csv -d $O/p2 -o run -- python3 tools/index_bench.py headline > $O/p2.log 2>&1 || exit 2
timeout -s KILL 200 rocprofv3 --pmc GRBM_GUI_ACTIVE --output-format csv -d $O/p3 -o run -- python3 tools/index_bench.py headline > $O/p3.log 2>&1 || exit 3
python3 - $O <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
  for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "k_idx_spec" in n or "k_idx_emit" in n or "k_decode<" in n or "k_idx_sync" in n:
      acc[n[:50]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
  print("==", k)
  for c, v in sorted(d.items()):
    print("  %-22s per dispatch %16.0f  (%d)" % (c, sum(v[1:]) / max(1, len(v) - 1), len(v)))
PY
