#!/bin/bash
# rocprofv3 records of bench.py workloads: a kernel-trace summary and separate
# FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md: one TCC counter group per
# pass), per workload.  usage: bash tools/profile_workloads.sh <outdir> [workload ...]
set -e
set -o pipefail
OUT=$1; shift
WL=${@:-headline headline_uniform trainer_round config2 config3 config4_share headline_c128 onebit onebit_c128}
export TMPDIR=/tmp
mkdir -p $OUT
for w in $WL; do
  A="--workload $w --no-cpu-baseline --steps 3 --warmup 1 --extra-steps 3"
  mkdir -p $OUT/$w
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$w/kt -o run -- python3 bench.py $A > $OUT/$w/kt.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$w/fetch -o run -- python3 bench.py $A > $OUT/$w/fetch.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$w/write -o run -- python3 bench.py $A > $OUT/$w/write.log 2>&1
  # keep the kernel stats and this package's counter rows only (the torch kernels' names
  # make the raw csv files tens of MB per pass)
  python3 - $OUT/$w <<'PY'
import csv, glob, os, sys
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
  os.remove(f)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
  with open(f) as fh:
    rows = list(csv.DictReader(fh))
  keep = [r for r in rows if "::k_" in r["Kernel_Name"]]
  with open(f, "w", newline="") as fh:
    w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()) if rows else ["Kernel_Name"])
    w.writeheader()
    w.writerows(keep)
PY
  echo "profiled $w"
done
echo PROFILE_DONE
