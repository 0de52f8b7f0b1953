# Decoder PMC passes (diagnostic): bash tools/diag/pmc_dec.sh <outdir> [lib]
set -e
export TMPDIR=/tmp
O=$1
LIB=${2:-}
mkdir -p $O
[ -n "$LIB" ] && export FEDCODEC_LIB=$LIB
C=256 timeout -k 10 120 python3 tools/dec_bench.py
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $O/p1 -o run -- python3 tools/dec_bench.py > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA --output-format csv -d $O/p2 -o run -- python3 tools/dec_bench.py > $O/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS --output-format csv -d $O/p3 -o run -- python3 tools/dec_bench.py > $O/p3.log 2>&1
python3 tools/summarize_pmc.py $O k_decode 2>&1 || true
