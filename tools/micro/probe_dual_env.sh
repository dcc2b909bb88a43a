mkdir -p gpurun_out
for e in "X=1" "GNNREC_RQ_CHUNK_FUSED=4" "GNNREC_RQ_CHUNK_FUSED=16" "GNNREC_RQ_CHUNK_FUSED=32" "X=1"; do
  echo -n "$e: " >> gpurun_out/dualenv.log
  env $e PROBE_DUAL=1 timeout -k 10 200 python tools/probe_c5.py 2>/dev/null | grep user >> gpurun_out/dualenv.log || exit 1
done
