mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then L=""; else L=tools/_diag/libgnnrec_$v.so; fi
  echo "== $v" >> gpurun_out/var.log
  GNNREC_LIB=${L:-gnn-recsys_amd/gnnrec/libgnnrec.so} PROBE_REL=bought-by PROBE_VARIANTS=${PV:-mfma} timeout -k 10 120 python tools/probe_c5.py >> gpurun_out/var.log 2>&1 || exit 1
done
