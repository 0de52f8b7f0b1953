#!/bin/bash
# round-5 V: (1) the N > 1 bench paths rehearsed on the final build -- 2 ranks on one
# device over gloo, 1024 x 25 M (each rank 512 clients: the eight-tile super-tile encoder),
# the headline sum bit-identical to N = 1; (2) PMC of the final k_encode2 per mode
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
D=$(mktemp -d)
export FEDCODEC_BENCH_BACKEND=gloo FEDCODEC_BENCH_ONE_DEVICE=1
timeout -k 10 400 python3 bench.py --gpus 2 --workload headline --clients 1024 --P 25000000 --steps 3 --warmup 1 --no-cpu-baseline --dump-result $D/sum_n2.npy > gpurun_out/r5v_n2.log 2>&1 || { tail -30 gpurun_out/r5v_n2.log; exit 1; }
grep -h '"n_gpus": 2' gpurun_out/r5v_n2.log | head -c 400; echo
unset FEDCODEC_BENCH_BACKEND FEDCODEC_BENCH_ONE_DEVICE
timeout -k 10 300 python3 bench.py --workload headline --clients 1024 --P 25000000 --steps 3 --warmup 1 --no-cpu-baseline --dump-result $D/sum_n1.npy > gpurun_out/r5v_n1.log 2>&1 || { tail -30 gpurun_out/r5v_n1.log; exit 1; }
python3 -c "import numpy as np; a=np.load('$D/sum_n1.npy'); b=np.load('$D/sum_n2.npy'); ok=bool((a.view(np.uint32)==b.view(np.uint32)).all()); print('N=2 vs N=1 dequantised sum identical:', a.shape, ok, float(np.abs(a).sum())); raise SystemExit(0 if ok else 1)" | tee gpurun_out/r5v_ident.txt || exit 1
rm -rf $D
O=gpurun_out/r5v_pmc; mkdir -p $O
for M in 1 0; do
C=1024 REPS=1 DEC=0 CAP=0.5 MODE=$M timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/m$M -o run -- python3 tools/enc_bench.py > $O/m$M.log 2>&1 || exit 1
python3 tools/summarize_pmc.py $O/m$M "k_encode2<" > $O/m$M.txt 2>&1 || true
cat $O/m$M.txt
find $O/m$M -name "*counter_collection.csv" -delete
done
