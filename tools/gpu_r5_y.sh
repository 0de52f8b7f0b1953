#!/bin/bash
# round-5 Y: decode_segment's loop unrolled by four (du: FC_DEC_UNROLL=1, batch points and
# arithmetic slots at fixed places), the lambda-restructured loop (current, not unrolled) and
# the previous commit (prev): decoder parity tests through du, then enc_bench decode times
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
FEDCODEC_LIB=federated_amd/libfedcodec_du.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_codec.py tests/test_gpu_configs.py tests/test_gpu_bare_decode.py tests/test_gpu_segmented.py > gpurun_out/r5y_tests.txt 2>&1 || { tail -30 gpurun_out/r5y_tests.txt; exit 1; }
tail -1 gpurun_out/r5y_tests.txt
O=gpurun_out/r5y.txt
: > $O
for rep in 1 2; do
  for L in federated_amd/libfedcodec_prev.so federated_amd/libfedcodec.so federated_amd/libfedcodec_du.so; do
    FEDCODEC_LIB=$L MODE=1 CAP=0.5 REPS=5 timeout -k 10 240 python3 tools/enc_bench.py 2>&1 | grep -v 'amdgpu.ids\|row bases' >> $O || exit 1
    FEDCODEC_LIB=$L MODE=1 C=128 P=1048576 STEP=0.007874015748031496 SIGMA=0.25 CAP=2 REPS=9 timeout -k 10 240 python3 tools/enc_bench.py 2>&1 | grep -v 'amdgpu.ids\|row bases' >> $O || exit 1
  done
done
cat $O
