#!/bin/bash
# round-5 B: full GPU suite (client-split passes), encoder floor (streaming form),
# copy variants, the new bench lines (bare_decode, config4_full) and the split lines
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5b_gputest.txt 2>&1 || exit 1
timeout -k 10 300 python3 tools/floor_bench.py > gpurun_out/r5b_floor.txt 2>&1 || exit 2
for v in "" _cpu8 _cpnt _cpu8nt _cpu2; do
  lib=federated_amd/libfedcodec$v.so
  FEDCODEC_LIB=$PWD/$lib timeout -k 10 120 python3 bench.py --workload copy > gpurun_out/r5b_copy$v.json 2>/dev/null || exit 3
done
for w in onebit_c128 onebit trainer_round bare_decode config4_full config4_share; do
  timeout -k 10 300 python3 bench.py --workload $w > gpurun_out/r5b_$w.json 2> gpurun_out/r5b_$w.err || exit 4
done
