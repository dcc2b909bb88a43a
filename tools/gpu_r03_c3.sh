#!/bin/bash
# C3 training step (d=128, mean_nn, 1024 pos x 2500 neg): probe at nw 0/2 and a kernel trace
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for nw in 0 2; do
  timeout -k 10 200 python -u tools/probe_c2_step.py 2500 $nw 128 mean_nn 2>/dev/null | tail -1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_c3 -o run -- python3 $R/tools/probe_c2_step.py 2500 0 128 mean_nn > $R/gpurun_out/r03_c3.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03_c3.log; exit 1; }
tail -1 $R/gpurun_out/r03_c3.log
