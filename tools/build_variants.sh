#!/bin/bash
# Diagnostic builds of libfedcodec: ablations (FC_ABL bits), phase stamps, occupancy.
set -e
cd "$(dirname "$0")/.."
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -fgpu-flush-denormals-to-zero -ffp-contract=off"
S=federated_amd/csrc/fedcodec.hip
for v in ${ABL:-1 2 4 8 15}; do /opt/rocm/bin/hipcc $F -DFC_ABL=$v -o federated_amd/libfedcodec_abl$v.so $S & done
/opt/rocm/bin/hipcc $F -DFC_STAMPS -o federated_amd/libfedcodec_stamps.so $S &
for w in ${WAVES:-4 6 8}; do /opt/rocm/bin/hipcc $F -DFC_ENC_WAVES=$w -o federated_amd/libfedcodec_w$w.so $S & done
wait
