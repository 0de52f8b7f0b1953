#!/bin/bash
# round-4 GPU batch 3: decoder chunk-size variants (16 / 32 / 64-byte lane loads): time and raw FETCH
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in "" _chunk2 _chunk4; do
  lib=federated_amd/libfedcodec$v.so
  echo "== $lib" >> gpurun_out/dec_chunk.txt
  FEDCODEC_LIB=$PWD/$lib C=1024 ITERS=4 timeout -k 10 200 python3 tools/dec_bench.py >> gpurun_out/dec_chunk.txt 2>&1 || exit 1
  FEDCODEC_LIB=$PWD/$lib C=1024 ITERS=2 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/dec_fetch$v -o run -- python3 tools/dec_bench.py > gpurun_out/dec_fetch$v.log 2>&1 || exit 2
done
