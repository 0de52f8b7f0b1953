# k_encode PMC at 128 vs 1024 clients (diagnostic): instructions per tile and VALU-pipe busy,
# to split the 128-client per-client penalty into extra work and extra waiting.
export TMPDIR=/tmp
O=/tmp/pmc_c128; mkdir -p $O gpurun_out
export MODE=${MODE:-1} REPS=1 DEC=0 FEDCODEC_ENC2=0
for C in 128 1024; do
  C=$C timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY --output-format csv -d $O/a$C -o run -- python3 tools/enc_bench.py > $O/a$C.log 2>&1 || { echo "pass a C=$C failed"; tail -5 $O/a$C.log; exit 1; }
  C=$C timeout -s KILL 150 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $O/b$C -o run -- python3 tools/enc_bench.py > $O/b$C.log 2>&1 || { echo "pass b C=$C failed"; tail -5 $O/b$C.log; exit 1; }
  echo "== C=$C"
  python3 tools/summarize_pmc.py $O/a$C "k_encode<" || true
  python3 tools/summarize_pmc.py $O/b$C "k_encode<" || true
done
