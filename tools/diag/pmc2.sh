set -e
export TMPDIR=/tmp
O=gpurun_out/pmc2; mkdir -p $O
export C=256 MODE=1 REPS=1
for E in 0 1; do
FEDCODEC_ENC2=$E timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH --output-format csv -d $O/e$E -o run -- python3 tools/enc_bench.py > $O/e$E.log 2>&1
done
python3 tools/summarize_pmc.py $O/e0 "k_encode<" || true
python3 tools/summarize_pmc.py $O/e1 "k_encode2<" || true
