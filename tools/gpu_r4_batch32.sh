#!/bin/bash
# round-4 GPU batch 32: config 2's quarter-tile decoder after the one-refill loop -- accumulator copies (1 / 2 default / 4),
# waves per SIMD (4 / 5 default / 6), lanes per tile (64 / 128 default / 256): decode parity subset, then dec_bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for v in; do  # (tests passed in the first run)
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_quarters.py tests/test_gpu_configs.py > gpurun_out/b32_$v.log 2>&1 || { echo "$v FAILED"; tail -30 gpurun_out/b32_$v.log; exit 1; }
  echo "$v tests: $(tail -1 gpurun_out/b32_$v.log)"
done
for rep in 1 2; do
  for v in "" _qrepl4 _qrepl1 _qwpe6; do
    a=$(FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=20 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1) || exit 2
    echo "lib$v | config2: $a"
  done
  for lpt in 64 256; do
    a=$(FEDCODEC_DEC_LPT=$lpt C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 ITERS=20 timeout -k 10 100 python3 tools/dec_bench.py 2>&1 | grep "decode" | tail -1) || exit 3
    echo "lib lanes/tile $lpt | config2: $a"
  done
done
for rep in 1 2; do for v in "" _qrepl4; do
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so timeout -k 10 200 python3 bench.py --workload config2 --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/b32_bench$v.json 2> gpurun_out/b32_bench$v.err || exit 4
  echo "lib$v bench config2: $(head -c 160 gpurun_out/b32_bench$v.json)"
done; done
