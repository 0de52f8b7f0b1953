#!/bin/bash
# Rehearsal of the N>1 bench paths on a 1-GPU box: 2 ranks on one device over gloo
# (stands in for RCCL).  `bench.py --gpus 2` starts its own 2 ranks (no torchrun on
# the command line); the headline round's dequantised sum must equal N=1 bit for
# bit; config 5's sharded one-bit round must run and print n_gpus 2.
# usage (GPU box): [GPUS=2 CLIENTS=64 P=2500000] bash tools/rehearse_multigpu.sh
# (CLIENTS=1024: each rank holds 512 clients, the super-tile encoder's N = 2 share;
# GPUS=4 CLIENTS=512 P=25000000: four ranks, each with the 8-GPU headline's 128-client share)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export FEDCODEC_BENCH_BACKEND=gloo FEDCODEC_BENCH_ONE_DEVICE=1
G=${GPUS:-2}
CL=${CLIENTS:-64}
PP=${P:-2500000}
timeout -k 10 300 python bench.py --gpus $G --workload headline --clients $CL --P $PP --steps 3 --warmup 1 --no-cpu-baseline --dump-result gpurun_out/sum_n2.npy > gpurun_out/rehearse2.log 2>&1 && echo REHEARSE_OK || { tail -30 gpurun_out/rehearse2.log; exit 1; }
grep -h "\"n_gpus\": $G" gpurun_out/rehearse2.log > /dev/null && echo N_GPUS_${G}_OK || { echo "no n_gpus $G line"; exit 1; }
timeout -k 10 300 python bench.py --gpus $G --workload onebit --clients $CL --P $PP --steps 3 --warmup 1 --dump-result gpurun_out/onebit_n2.npy > gpurun_out/rehearse2_onebit.log 2>&1 && echo ONEBIT2_OK || { tail -30 gpurun_out/rehearse2_onebit.log; exit 1; }
unset FEDCODEC_BENCH_BACKEND FEDCODEC_BENCH_ONE_DEVICE
timeout -k 10 300 python bench.py --workload headline --clients $CL --P $PP --steps 3 --warmup 1 --no-cpu-baseline --dump-result gpurun_out/sum_n1.npy > gpurun_out/rehearse1.log 2>&1 && echo N1_OK || { tail -30 gpurun_out/rehearse1.log; exit 1; }
python -c "import numpy as np; a=np.load('gpurun_out/sum_n1.npy'); b=np.load('gpurun_out/sum_n2.npy'); ok=bool((a.view(np.uint32)==b.view(np.uint32)).all()); print('identical', a.shape, ok, float(np.abs(a).sum())); raise SystemExit(0 if ok else 1)"
