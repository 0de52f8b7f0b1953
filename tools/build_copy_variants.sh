#!/bin/bash
# Diagnostic builds of libfedcodec for the copy-kernel A/B (FC_COPY_U loads in flight
# per lane, FC_COPY_NT non-temporal, FC_COPY_WG workgroups per CU).
set -e
cd "$(dirname "$0")/.."
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fgpu-flush-denormals-to-zero -ffp-contract=off -fno-slp-vectorize -mllvm -amdgpu-atomic-optimizer-strategy=None"
S=federated_amd/csrc/fedcodec.hip
/opt/rocm/bin/hipcc $F -DFC_COPY_U=8 -o federated_amd/libfedcodec_cpu8.so $S &
/opt/rocm/bin/hipcc $F -DFC_COPY_NT=1 -o federated_amd/libfedcodec_cpnt.so $S &
/opt/rocm/bin/hipcc $F -DFC_COPY_U=8 -DFC_COPY_NT=1 -o federated_amd/libfedcodec_cpu8nt.so $S &
/opt/rocm/bin/hipcc $F -DFC_COPY_U=2 -DFC_COPY_WG=16 -o federated_amd/libfedcodec_cpu2.so $S &
wait
