# Encoder PMC at the headline size with four-tile tickets (diagnostic): instructions and
# busy cycles of k_encode2 per mode.  Writes gpurun_out/pmc4/.
set -e
export TMPDIR=/tmp
O=gpurun_out/pmc4; mkdir -p $O
export C=${C:-1024} REPS=1 DEC=0 FEDCODEC_ENC2=1 FEDCODEC_ENC_NT=4
for M in 1 0; do
MODE=$M timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/m$M -o run -- python3 tools/enc_bench.py > $O/m$M.log 2>&1
python3 tools/summarize_pmc.py $O/m$M "k_encode2<" || true
done
