#!/bin/bash
# time k_encode for each diagnostic build (tools/build_variants.sh), back to back
for v in ${VARIANTS:-base abl1 abl2 abl4 abl8 abl15}; do
  if [ $v = base ]; then lib=federated_amd/libfedcodec.so; else lib=federated_amd/libfedcodec_$v.so; fi
  echo -n "$v: "; FEDCODEC_LIB=$lib C=${C:-1024} P=${P:-6000000} MODE=${MODE:-1} timeout -k 10 120 python tools/stamps.py 2>&1 | grep encode | tail -1
done
