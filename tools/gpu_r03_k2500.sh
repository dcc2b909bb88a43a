#!/bin/bash
# C2 at the reference's K = 2500: kernel trace
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_k2500 -o run -- python3 $R/tools/probe_c2_step.py 2500 0 > $R/gpurun_out/r03_k2500.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03_k2500.log; exit 1; }
tail -1 $R/gpurun_out/r03_k2500.log
