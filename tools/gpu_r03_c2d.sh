#!/bin/bash
# C2 kernel traces at num_workers 0 and 2 (fused batch head): GPU time and busy fraction
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for nw in 0 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_c2d_nw$nw -o run -- python3 $R/tools/probe_c2_step.py 10 $nw > $R/gpurun_out/r03_c2d_nw$nw.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03_c2d_nw$nw.log; exit 1; }
  tail -1 $R/gpurun_out/r03_c2d_nw$nw.log
done
echo traces ok
