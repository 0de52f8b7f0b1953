#!/bin/bash
# round-5 K: k_encode2 ablations with eight-tile tickets (FC_ABL builds, one input set) and
# its PMC per mode (1024 x 25 M)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
L="federated_amd/libfedcodec_base.so federated_amd/libfedcodec_abl1.so federated_amd/libfedcodec_abl2.so federated_amd/libfedcodec_abl4.so federated_amd/libfedcodec_abl8.so federated_amd/libfedcodec_abl64.so federated_amd/libfedcodec_base.so"
LIBS="$L" CAP=0.5 REPS=5 timeout -k 10 500 python3 -u tools/diag/enc_ablate.py 2>&1 | grep -v amdgpu.ids > gpurun_out/r5k_abl.txt || exit 1
cat gpurun_out/r5k_abl.txt
O=gpurun_out/r5k_pmc; mkdir -p $O
for M in 1 0; do
C=1024 REPS=1 DEC=0 CAP=0.5 MODE=$M timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/m$M -o run -- python3 tools/enc_bench.py > $O/m$M.log 2>&1 || exit 1
python3 tools/summarize_pmc.py $O/m$M "k_encode2<" || true
done
