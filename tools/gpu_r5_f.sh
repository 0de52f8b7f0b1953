#!/bin/bash
# round-5 F: k_encode2 knob A/B on one box -- v0: no scalar round-2 xor, no fresh
# arguments; v1: + round-2 xor; v2: + partials / index pointers re-read; current: +
# status pointer and T2 re-read.  Then the streaming floor with one / two tiles in flight.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for m in 1 1 0; do
  for v in _v0 _v1 _v2 ""; do
    FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so CAP=0.6 MODE=$m REPS=5 DEC=0 timeout -k 10 200 python3 tools/enc_bench.py >> gpurun_out/r5f_enc.txt 2>&1 || exit 2
  done
done
timeout -k 10 200 python3 tools/floor_bench.py > gpurun_out/r5f_floor.txt 2>&1 || exit 3
FEDCODEC_FLOOR_DEPTH=2 timeout -k 10 200 python3 tools/floor_bench.py > gpurun_out/r5f_floor_d2.txt 2>&1 || exit 4
