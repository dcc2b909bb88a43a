#!/bin/bash
# round 5 (t): GPU occupancy of the captured C2 loop (K = 10): a kernel trace summarised on
# the box by tools/rocpd_timeline.py (busy fraction, idle gaps, per-queue time)
set -o pipefail
O=gpurun_out/r05t
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for K in 10 2500; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl$K -o tl -- python3 $R/tools/probe_captured_loop.py $K 100 > $R/$O/loop$K.json 2> $R/$O/loop$K.err || { echo "trace $K failed"; tail -20 $R/$O/loop$K.err; exit 1; }
  cat $R/$O/loop$K.json
  python3 $R/tools/rocpd_timeline.py $(ls /tmp/tl$K/*.db /tmp/tl$K/*/*.db 2>/dev/null | head -1) > $R/$O/timeline$K.json && cat $R/$O/timeline$K.json
done
