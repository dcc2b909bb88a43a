#!/bin/bash
# probe_c5.py's dual (user-side) measurement over libgnnrec variants: VARIANTS="default u8"
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then L=gnn-recsys_amd/gnnrec/libgnnrec.so; else L=tools/_diag/libgnnrec_$v.so; fi
  echo -n "$v: " >> gpurun_out/dualvar.log
  GNNREC_LIB=$L PROBE_DUAL=1 timeout -k 10 200 python tools/probe_c5.py 2>/dev/null | grep user >> gpurun_out/dualvar.log || exit 1
done
