#!/bin/bash
# PMC passes for k_encode / k_decode (each counter group in its own run, no tracing domains).
# usage: bash tools/prof_counters.sh <outdir> -- <cmd...>
set -e
OUT=$1; shift; shift
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- "$@" > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/p1 -o run -- "$@" > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p2 -o run -- "$@" > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p3 -o run -- "$@" > $OUT/p3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/p4 -o run -- "$@" > $OUT/p4.log 2>&1
echo PROF_DONE
