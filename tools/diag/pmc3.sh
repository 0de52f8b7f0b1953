# Encoder PMC at the headline size (diagnostic): VALU-pipe busy vs wave cycles for k_encode2 / k_encode.
set -e
export TMPDIR=/tmp
O=gpurun_out/pmc3; mkdir -p $O
export C=${C:-1024} MODE=${MODE:-1} REPS=1
for E in 1 0; do
FEDCODEC_ENC2=$E timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d $O/e$E -o run -- python3 tools/enc_bench.py > $O/e$E.log 2>&1
done
python3 tools/summarize_pmc.py $O/e1 "k_encode2<" || true
python3 tools/summarize_pmc.py $O/e0 "k_encode<" || true
