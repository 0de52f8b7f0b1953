# decoder segment span A/B (headline density, 1024 clients; config 3; config 2) with lanes per tile
set -o pipefail
cd $GRAFT_REPO_ROOT
for L in federated_amd/libfedcodec.so federated_amd/libfedcodec_span2.so federated_amd/libfedcodec_span4.so; do
  for lpt in 128 256; do
    for cfg in "C=1024 P=25000000 STEP=0.5 SIGMA=1.0" "C=256 P=4050748 STEP=1.0 SIGMA=1.0" "C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25"; do
      echo "== $L lpt=$lpt $cfg"
      env $cfg ITERS=3 FEDCODEC_DEC_LPT=$lpt FEDCODEC_LIB=$L timeout -k 10 150 python -u tools/dec_bench.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done
