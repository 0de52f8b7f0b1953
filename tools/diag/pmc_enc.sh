# Encoder PMC passes (diagnostic): bash tools/diag/pmc_enc.sh <outdir> <mode>
set -e
export TMPDIR=/tmp
O=$1; M=${2:-1}
mkdir -p $O
export C=256 MODE=$M REPS=1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $O/p1 -o run -- python3 tools/enc_bench.py > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA --output-format csv -d $O/p2 -o run -- python3 tools/enc_bench.py > $O/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM --output-format csv -d $O/p3 -o run -- python3 tools/enc_bench.py > $O/p3.log 2>&1
python3 tools/summarize_pmc.py $O "k_encode<" 2>&1 || true
