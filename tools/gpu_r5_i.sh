#!/bin/bash
# round-5 I: per-ticket cost of k_encode2 -- two- vs four-tile tickets (FEDCODEC_ENC_NT), 1024 x 25 M
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5i.txt
: > $O
for m in 1 0; do
  for nt in 2 4; do
    FEDCODEC_ENC_NT=$nt MODE=$m CAP=0.6 DEC=0 REPS=5 timeout -k 10 240 python3 tools/enc_bench.py 2>&1 | grep -v amdgpu.ids | sed "s/^/NT=$nt /" >> $O || exit 1
  done
done
cat $O
