#!/bin/bash
# round 4 (k): kernel trace of the K = 2500 C2 step (23 steps: 3 warm-up + 20 timed) on the
# current sources — per-kernel totals and dispatch counts, for the launch-count / fusion work
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04k
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o k2500 -- python3 $R/tools/probe_c2_step.py 2500 2 \
  > $O/k2500_prof.log 2>&1 || { echo "k2500 trace failed"; tail -5 $O/k2500_prof.log; exit 1; }
tail -1 $O/k2500_prof.log | cut -c1-300
db=$(find $O/prof -name '*results.db' | head -1)
python3 $R/tools/rocpd_summary.py "$db" 40 > $O/k2500_kernel_stats.md && head -3 $O/k2500_kernel_stats.md
