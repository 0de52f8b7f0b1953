#!/bin/bash
# round-4 GPU batch 9: WRITE_SIZE calibration of the encoder's store pattern
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/wcal
mkdir -p $O
timeout -k 10 60 ./tools/microbench/write_calib > $O/times.txt 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- ./tools/microbench/write_calib > $O/w.log 2>&1 || exit 2
cat $O/times.txt
python3 - $O/w <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
  for r in csv.DictReader(open(f)):
    print("%-60s WRITE_SIZE %.4f GB" % (r["Kernel_Name"][:60], float(r["Counter_Value"]) * 1024 / 1e9))
PY
