#!/bin/bash
# round 4 (p): is the K = 10 C2 step host- or GPU-bound on the final tree?  kernel trace of the
# probe (sampling thread) -> GPU busy fraction of the timed steps; host-op breakdown (torch
# profiler, CPU activity only, no sampling thread)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04p
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o k10 -- python3 $R/tools/probe_c2_step.py 10 2 \
  > $O/k10_trace.log 2>&1 || { echo "trace failed"; tail -5 $O/k10_trace.log; exit 1; }
W=$(tail -1 $O/k10_trace.log | grep -o "'wall_ms_per_step': [0-9.]*" | grep -o "[0-9.]*$")
echo "wall $W"
python3 $R/tools/c2_busy.py $(find $O/trace -name '*kernel_trace.csv' | head -1) $W 20 | head -30
cd $R && timeout -k 10 300 python3 tools/profile_c2_torch.py 10 0 > $O/k10_host.txt 2>&1 || { echo "host profile failed"; tail -5 $O/k10_host.txt; exit 1; }
head -40 $O/k10_host.txt | cut -c1-200
