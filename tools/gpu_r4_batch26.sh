#!/bin/bash
# round-4 GPU batch 26: decoder knob builds (waves/SIMD 6, batch points every 2 / 8 iterations, early long-code slot
# at 8 waiting lanes) against the default: decode parity subset, then dec_bench at config 2 and the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in wpe6 batch2 batch8 ll8; do
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_codec.py tests/test_gpu_quarters.py > gpurun_out/b26_$v.log 2>&1 || { echo "$v FAILED"; tail -5 gpurun_out/b26_$v.log; continue; }
  echo "$v tests: $(tail -1 gpurun_out/b26_$v.log)"
done
for rep in 1 2; do for v in "" _wpe6 _batch2 _batch8 _ll8; do
  L=$PWD/federated_amd/libfedcodec$v.so
  a=$(FEDCODEC_LIB=$L C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=6 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1)
  b=$(FEDCODEC_LIB=$L C=1024 ITERS=3 timeout -k 10 150 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1)
  c=$(FEDCODEC_LIB=$L C=128 ITERS=4 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1)
  echo "lib$v | config2: $a | headline: $b | 128x25M: $c"
done; done
