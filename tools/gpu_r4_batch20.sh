#!/bin/bash
# round-4 GPU batch 20: decoder knobs at the 8-GPU share (128 x 25 M): lanes per unit, span, grid
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for rep in 1 2; do
for kv in "X=0" "FEDCODEC_DEC_LPT=64" "FEDCODEC_DEC_LPT=256" "FEDCODEC_DEC_SPAN=2" "FEDCODEC_DEC_GRID=768" "FEDCODEC_DEC_GRID=2048"; do
  env $kv timeout -k 10 200 python3 bench.py --workload headline_c128 --no-cpu-baseline --steps 5 --warmup 2 --extra-steps 5 > gpurun_out/k.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/k.json').read().strip().splitlines()[-1]); print('%-22s step %.3f  encode %.3f  decode %.3f' % ('$kv', d['ms_per_step'], d['roofline']['launch_ms'], d['decode']['launch_ms']))"
done; done
