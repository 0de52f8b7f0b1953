#!/bin/bash
# round-4 GPU batch 18: the N>1 bench paths rehearsed on one card (2 ranks over gloo) on the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash tools/rehearse_multigpu.sh > gpurun_out/rehearse_r4.txt 2>&1 || { cat gpurun_out/rehearse_r4.txt; exit 1; }
cat gpurun_out/rehearse_r4.txt
grep -h '"n_gpus"' gpurun_out/rehearse2.log gpurun_out/rehearse2_onebit.log gpurun_out/rehearse1.log >> gpurun_out/rehearse_r4.txt
CLIENTS=1024 P=25000000 bash tools/rehearse_multigpu.sh > gpurun_out/rehearse_r4_1024.txt 2>&1 || { cat gpurun_out/rehearse_r4_1024.txt; exit 2; }
cat gpurun_out/rehearse_r4_1024.txt
grep -h '"n_gpus"' gpurun_out/rehearse2.log gpurun_out/rehearse2_onebit.log gpurun_out/rehearse1.log >> gpurun_out/rehearse_r4_1024.txt
