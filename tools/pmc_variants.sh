#!/bin/bash
# Instruction-mix counters of k_encode for each diagnostic build (tools/build_variants.sh).
# usage: bash tools/pmc_variants.sh <outdir> [variants...]
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
for v in "$@"; do
  if [ $v = base ]; then lib=federated_amd/libfedcodec.so; else lib=federated_amd/libfedcodec_$v.so; fi
  FEDCODEC_LIB=$lib timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/$v/p1 -o run -- python3 tools/stamps.py > $OUT/$v.p1.log 2>&1 || exit 1
  FEDCODEC_LIB=$lib timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/$v/p2 -o run -- python3 tools/stamps.py > $OUT/$v.p2.log 2>&1 || exit 1
  echo "== $v"; python3 tools/summarize_pmc.py $OUT/$v k_encode
done
