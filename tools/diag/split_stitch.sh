# split stitch A/B: bench workloads with the stitch in order or on a second stream
# (copy workgroups per CU 1 / 2 / 4 / 16)
cd $GRAFT_REPO_ROOT
for w in ${WL:-headline_c128 config3 config4_share}; do
  for cfg in "FEDCODEC_SPLIT_STITCH=0" "FEDCODEC_SPLIT_COPY_WG=1" "FEDCODEC_SPLIT_COPY_WG=2" "FEDCODEC_SPLIT_COPY_WG=4" "FEDCODEC_SPLIT_COPY_WG=16"; do
    env $cfg timeout -k 10 200 python bench.py --workload $w 2>/dev/null | python -c "
import sys, json
j = json.loads(sys.stdin.read().strip().splitlines()[-1])
print('%-14s %-26s step %.3f  encode %.3f  decode %.3f' % ('$w', '$cfg', j['ms_per_step'], j['roofline']['launch_ms'], j['decode']['launch_ms']))" || exit 1
  done
done
