#!/bin/bash
# round 5 (i): kernel trace of the captured C2 step (K = 10, then K = 2500), summarised on the
# box (the databases stay there)
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for K in 10 2500; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tr$K -o cap -- python3 $GRAFT_REPO_ROOT/tools/probe_captured_step.py --captured-only $K > $GRAFT_REPO_ROOT/$O/probe$K.json 2> $GRAFT_REPO_ROOT/$O/probe$K.err || { echo "trace $K failed"; tail -20 $GRAFT_REPO_ROOT/$O/probe$K.err; exit 1; }
  cat $GRAFT_REPO_ROOT/$O/probe$K.json
  python3 $GRAFT_REPO_ROOT/tools/rocpd_stats.py $(ls /tmp/tr$K/*.db /tmp/tr$K/*/*.db 2>/dev/null | head -1) > $GRAFT_REPO_ROOT/$O/kernels$K.csv
  head -30 $GRAFT_REPO_ROOT/$O/kernels$K.csv | cut -c1-110
done
