#!/bin/bash
# round 4 (g): where the reference-default C2 step (K = 2500 negatives) spends its time on the
# current sources: probe at num_workers 2 and 0, kernel trace (nw 0) + busy summary
set -o pipefail
mkdir -p gpurun_out/r04g
O=$GRAFT_REPO_ROOT/gpurun_out/r04g
R=$GRAFT_REPO_ROOT
for nw in 2 0; do
  timeout -k 10 200 python -u tools/probe_c2_step.py 2500 $nw > $O/probe_nw$nw.log 2>&1 || { echo "probe failed"; tail $O/probe_nw$nw.log; exit 1; }
  tail -1 $O/probe_nw$nw.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/tools/probe_c2_step.py 2500 0 > $O/trace.log 2>&1 || { echo "trace failed"; tail $O/trace.log; exit 1; }
W=$(grep wall_ms $O/trace.log | tail -1 | python3 -c "import sys,ast; print(ast.literal_eval(sys.stdin.read())['wall_ms_per_step'])")
python3 $R/tools/c2_busy.py $(find $O/trace -name '*kernel_trace.csv' | head -1) $W > $O/busy.txt && head -40 $O/busy.txt
