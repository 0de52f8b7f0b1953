#!/bin/bash
# Rehearsal of the N>1 bench path on a 1-GPU box: 2 ranks on one device over gloo
# (stands in for RCCL), then the same round at N=1; the dequantised sums must match bit for bit.
# usage (GPU box): bash tools/rehearse_multigpu.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# 2-rank rehearsal of the multi-GPU bench path on one device (gloo stands in for RCCL):
# the round's dequantised sum must equal the 1-rank result bit for bit
FEDCODEC_BENCH_BACKEND=gloo FEDCODEC_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --clients 64 --P 2500000 --steps 3 --warmup 1 --no-cpu-baseline --dump-result gpurun_out/sum_n2.npy > gpurun_out/rehearse2.log 2>&1 && echo REHEARSE_OK || { tail -30 gpurun_out/rehearse2.log; exit 1; }
timeout -k 10 300 python bench.py --clients 64 --P 2500000 --steps 3 --warmup 1 --no-cpu-baseline --dump-result gpurun_out/sum_n1.npy > gpurun_out/rehearse1.log 2>&1 && echo N1_OK || { tail -30 gpurun_out/rehearse1.log; exit 1; }
python -c "import numpy as np; a=np.load('gpurun_out/sum_n1.npy'); b=np.load('gpurun_out/sum_n2.npy'); print('identical', a.shape, bool((a.view(np.uint32)==b.view(np.uint32)).all()), float(np.abs(a).sum()))"
