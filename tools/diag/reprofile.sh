# re-profile workloads into gpurun_out/prof_rec (small files only) and run the default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_rec
bash tools/profile_workloads.sh /tmp/prof $WL > gpurun_out/prof_rec/profile.log 2>&1 || { tail -20 gpurun_out/prof_rec/profile.log; exit 1; }
python3 tools/make_profile_record.py /tmp/prof gpurun_out/prof_rec $WL > gpurun_out/prof_rec/record.log 2>&1 || { tail -20 gpurun_out/prof_rec/record.log; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/prof_rec/bench_line.json 2> gpurun_out/prof_rec/bench.err || exit 1
ls gpurun_out/prof_rec
