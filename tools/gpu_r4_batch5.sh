#!/bin/bash
# round-4 GPU batch 5: decoder SQ/TCC counters at the headline (1024 x 25 M), async 16-B lane loads
# (default) vs whole 64-B chunks (FC_DEC_CHUNK=4): is the decoder issue-bound or fetch-bound?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp C=1024 ITERS=2
for v in "" _chunk4; do
  O=gpurun_out/pmc_dec$v
  mkdir -p $O
  export FEDCODEC_LIB=$PWD/federated_amd/libfedcodec$v.so
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $O/p1 -o run -- python3 tools/dec_bench.py > $O/p1.log 2>&1 || exit 1
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS --output-format csv -d $O/p2 -o run -- python3 tools/dec_bench.py > $O/p2.log 2>&1 || exit 2
  timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p3 -o run -- python3 tools/dec_bench.py > $O/p3.log 2>&1 || exit 3
  python3 tools/summarize_pmc.py $O k_decode > $O/summary.txt 2>&1 || true
done
echo BATCH5_DONE
