#!/bin/bash
# round-4 GPU batch 33: two accumulator copies for the main (whole-tile) decoder segments (FC_DEC_REPL=2) against one
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
FEDCODEC_LIB=$PWD/federated_amd/libfedcodec_repl2.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_codec.py tests/test_gpu_decoder_span.py tests/test_gpu_configs.py > gpurun_out/b33_tests.log 2>&1 || { tail -30 gpurun_out/b33_tests.log; exit 1; }
echo "repl2 tests: $(tail -1 gpurun_out/b33_tests.log)"
for rep in 1 2; do for v in "" _repl2; do
  L=$PWD/federated_amd/libfedcodec$v.so
  a=$(FEDCODEC_LIB=$L C=1024 ITERS=5 timeout -k 10 150 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1) || exit 2
  b=$(FEDCODEC_LIB=$L C=128 ITERS=8 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1) || exit 3
  c=$(FEDCODEC_LIB=$L C=256 P=4050748 STEP=1.0 ITERS=10 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1) || exit 4
  echo "lib$v | headline: $a | 128x25M: $b | 256x4M step 1: $c"
done; done
