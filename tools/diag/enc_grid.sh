# k_encode at 128 clients (one GPU's share of the 8-GPU headline): encode time against
# the persistent grid (waves; default = occupancy) and the look-back prefetch window
set -o pipefail
cd $GRAFT_REPO_ROOT
for g in 1024 2048 3072 0; do
  for w in 16 64; do
    if [ $g = 0 ]; then unset FEDCODEC_ENC_GRID; else export FEDCODEC_ENC_GRID=$g; fi
    echo "grid=$g lbwin=$w" >> gpurun_out/enc_grid.log
    FEDCODEC_LB_WIN=$w C=128 DEC=0 REPS=7 timeout -k 10 100 python -u tools/enc_bench.py >> gpurun_out/enc_grid.log 2>&1 || exit 1
  done
done
