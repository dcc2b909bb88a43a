#!/bin/bash
# round 5 (ab): GPU occupancy of the captured C2 loop on the current tree — K = 10 (provable
# capacities) and K = 2500 (learned): kernel traces summarised on the box
# (tools/rocpd_timeline.py: busy fraction between the loop's marker kernels, idle gaps)
set -o pipefail
O=gpurun_out/r05ab
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for spec in "10 provable" "2500 auto"; do
  set -- $spec
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl$1 -o tl -- python3 $R/tools/probe_captured_loop.py $1 100 0 2 $2 > $R/$O/loop$1.json 2> $R/$O/loop$1.err || { echo "trace $1 failed"; tail -20 $R/$O/loop$1.err; exit 1; }
  cat $R/$O/loop$1.json
  python3 $R/tools/rocpd_timeline.py $(ls /tmp/tl$1/*.db /tmp/tl$1/*/*.db 2>/dev/null | head -1) > $R/$O/timeline$1.json && cat $R/$O/timeline$1.json
done
