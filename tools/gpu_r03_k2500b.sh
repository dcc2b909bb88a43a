#!/bin/bash
# C2 at the reference's K = 2500 and at K = 10 (fused Adam): kernel traces + busy fraction
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for K in 2500 10; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03e_k$K -o run -- python3 $R/tools/probe_c2_step.py $K 0 > $R/gpurun_out/r03e_k$K.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03e_k$K.log; exit 1; }
  tail -1 $R/gpurun_out/r03e_k$K.log
  W=$(tail -1 $R/gpurun_out/r03e_k$K.log | python3 -c "import sys,ast; print(ast.literal_eval(sys.stdin.read())['wall_ms_per_step'])")
  python3 $R/tools/c2_busy.py $(find $R/gpurun_out/r03e_k$K -name '*kernel_trace.csv' | head -1) $W > $R/gpurun_out/r03e_k${K}_busy.txt && head -30 $R/gpurun_out/r03e_k${K}_busy.txt
done
