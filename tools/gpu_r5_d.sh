#!/bin/bash
# round-5 D: packed-pair quantiser / distortion + round-2 Philox xor (current) against
# the nonzero-mask build (libfedcodec_nz.so), one box; encoder parity suites first
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_supertile.py tests/test_gpu_configs.py tests/test_gpu_segmented.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5d_tests.txt 2>&1 || exit 1
for m in 1 0; do
  for v in _nz "" _nz ""; do
    FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so CAP=0.6 MODE=$m REPS=5 DEC=0 timeout -k 10 200 python3 tools/enc_bench.py >> gpurun_out/r5d_enc.txt 2>&1 || exit 2
  done
done
