#!/bin/bash
# round-4 GPU batch 12: aux_bench (with the bare-string index rebuild line), index rebuild kernel split per workload
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/aux_bench.py > gpurun_out/aux_bench_r4.txt 2>&1 || { tail -20 gpurun_out/aux_bench_r4.txt; exit 1; }
cat gpurun_out/aux_bench_r4.txt
for w in headline config2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/idxsplit_$w -o run -- python3 tools/index_bench.py $w > gpurun_out/idxsplit_$w.log 2>&1 || exit 2
  rm -f gpurun_out/idxsplit_$w/*kernel_trace.csv
  grep -h "k_idx\|k_decode" gpurun_out/idxsplit_$w/*kernel_stats.csv | cut -d, -f1-4
done
for rep in 1 2; do for w in 4 6 8; do
  echo "== emit waves/SIMD $w" >> gpurun_out/idx_emit_wpe.txt
  FEDCODEC_LIB=$PWD/federated_amd/libfedcodec_emit$w.so timeout -k 10 200 python3 tools/index_bench.py >> gpurun_out/idx_emit_wpe.txt 2>&1 || exit 3
done; done
grep -v amdgpu.ids gpurun_out/idx_emit_wpe.txt
