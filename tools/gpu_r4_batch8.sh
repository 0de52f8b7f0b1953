#!/bin/bash
# round-4 GPU batch 8: line-aligned code stores, one-instruction metadata stores, paired status
# granules (+ XCD-group ticket streams, knob FEDCODEC_XCD_SHARD): GPU suite, step times against
# the previous build (libfedcodec_base.so), encoder WRITE_SIZE
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/st
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B=$PWD/federated_amd/libfedcodec_base.so
N=$PWD/federated_amd/libfedcodec.so
for rep in 1 2; do for v in "base:$B:1" "new:$N:1" "new_noxcd:$N:0"; do
  IFS=: read name lib x <<< "$v"
  for w in headline headline_uniform config2 config3 headline_c128; do
    FEDCODEC_LIB=$lib FEDCODEC_XCD_SHARD=$x timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --steps 5 --warmup 2 --extra-steps 5 > $O/b_${w}_$name.json 2> $O/b_${w}_$name.err || exit 2
    python3 -c "
import json
d = json.loads(open('$O/b_${w}_$name.json').read().strip().splitlines()[-1])
print('%-10s %-18s step %.3f ms  encode %.3f ms  decode %s' % ('$name', '$w', d['ms_per_step'], d['roofline']['launch_ms'], d.get('decode', {}).get('launch_ms')), flush=True)
" | tee -a $O/ab.txt
  done
done; done
for v in "base:$B" "new:$N"; do
  IFS=: read name lib <<< "$v"
  for w in headline config2; do
    FEDCODEC_LIB=$lib timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_${w}_$name -o run -- python3 bench.py --workload $w --no-cpu-baseline --steps 2 --warmup 1 --extra-steps 2 > $O/write_${w}_$name.log 2>&1 || exit 3
    python3 - $O/write_${w}_$name $name $w <<'PY' | tee -a $O/write.txt
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
  for r in csv.DictReader(open(f)):
    acc[r["Kernel_Name"][:50]].append(float(r["Counter_Value"]))
for k, v in acc.items():
  if "k_encode" in k: print("%-5s %-9s %-50s WRITE_SIZE per launch %.4f GB" % (sys.argv[2], sys.argv[3], k, sum(v) / len(v) * 1024 / 1e9))
PY
  done
done
echo BATCH8_DONE
