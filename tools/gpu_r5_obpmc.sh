#!/bin/bash
# round-5 OBPMC: SQ counters of k_mask_encode (one-bit share, 128 x 25 M) beside k_client_norms (trainer round,
# 128 clients): is the mask encoder issue-bound?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/obpmc && mkdir -p gpurun_out/obpmc
for w in onebit_c128 trainer_round_c128; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/obpmc/$w -o run -- python3 bench.py --workload $w --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/obpmc/$w.log 2>&1 || { tail -5 gpurun_out/obpmc/$w.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for w in ["onebit_c128", "trainer_round_c128"]:
  f = glob.glob("gpurun_out/obpmc/%s/**/*counter_collection.csv" % w, recursive=True)[0]
  acc = collections.defaultdict(lambda: collections.defaultdict(list))
  for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "k_mask_encode" in n or "k_client_norms" in n:
      acc[n.split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
  for k, d in acc.items():
    print(w, k)
    for c, v in sorted(d.items()):
      print("   %-22s mean %.4g  n %d" % (c, sum(v) / len(v), len(v)))
PY
find gpurun_out/obpmc -name "*.csv" -size +2M -delete
