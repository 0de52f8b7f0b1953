#!/bin/bash
# round-4 GPU batch 30: the quarter-tile LONG loop refilling once per iteration (FC_DEC_LONG_R1) at 2 / 3 / 4 codes
# per iteration, and 3 codes per iteration without it, against the default: decode parity subset, then dec_bench at
# config 2 (dense 8-bit-step streams, the LONG loop) and the headline
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in r1u2 r1u3 r1u4 u3; do
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_codec.py tests/test_gpu_quarters.py tests/test_gpu_configs.py tests/test_gpu_edge_cases.py > gpurun_out/b30_$v.log 2>&1 || { echo "$v FAILED"; tail -30 gpurun_out/b30_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/b30_$v.log)"
done
for rep in 1 2; do for v in "" _r1u2 _r1u3 _r1u4 _u3; do
  L=$PWD/federated_amd/libfedcodec$v.so
  a=$(FEDCODEC_LIB=$L C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=6 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1) || exit 2
  b=$(FEDCODEC_LIB=$L C=1024 ITERS=3 timeout -k 10 150 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1) || exit 3
  echo "lib$v | config2: $a | headline: $b"
done; done
for v in "" _r1u3; do
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so timeout -k 10 200 python3 bench.py --workload config2 --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/b30_bench$v.json 2> gpurun_out/b30_bench$v.err || exit 4
  echo "lib$v bench config2: $(head -c 400 gpurun_out/b30_bench$v.json)"
done
