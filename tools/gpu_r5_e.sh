#!/bin/bash
# round-5 E: fewer SGPRs held across k_encode2's ticket loop (once-per-ticket fields
# re-read from the kernel arguments) against the nonzero-mask build, one box; the
# streaming floor with one / two tiles in flight per wave
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for m in 1 0; do
  for v in _nz "" _nz "" _nz ""; do
    FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so CAP=0.6 MODE=$m REPS=5 DEC=0 timeout -k 10 200 python3 tools/enc_bench.py >> gpurun_out/r5e_enc.txt 2>&1 || exit 2
  done
done
timeout -k 10 200 python3 tools/floor_bench.py > gpurun_out/r5e_floor.txt 2>&1 || exit 3
FEDCODEC_FLOOR_DEPTH=2 timeout -k 10 200 python3 tools/floor_bench.py > gpurun_out/r5e_floor_d2.txt 2>&1 || exit 4
