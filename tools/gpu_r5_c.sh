#!/bin/bash
# round-5 C: encoder A/B on one box (round-4 source vs the nonzero mask from the
# chained pair table), stochastic and uniform, four-tile tickets (CAP 0.6 B/elt);
# the streaming floor at the encoder's occupancy (4 waves / SIMD)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for m in 1 0; do
  for v in _base "" _base ""; do
    FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so CAP=0.6 MODE=$m REPS=5 timeout -k 10 200 python3 tools/enc_bench.py >> gpurun_out/r5c_enc.txt 2>&1 || exit 1
  done
done
timeout -k 10 200 python3 tools/floor_bench.py > gpurun_out/r5c_floor.txt 2>&1 || exit 2
FEDCODEC_FLOOR_LDS=40960 timeout -k 10 200 python3 tools/floor_bench.py > gpurun_out/r5c_floor_occ4.txt 2>&1 || exit 3
