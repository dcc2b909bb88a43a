#!/bin/bash
# round 5 (ad): occupancy of the eager K = 2500 C2 loop (sampling thread on its own stream):
# busy fraction and per-queue kernel time between the loop's marker kernels
set -o pipefail
O=gpurun_out/r05ad
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/et -o et -- python3 $R/tools/probe_eager_step.py 2500 60 > $R/$O/eager.json 2> $R/$O/eager.err || { echo "trace failed"; tail -20 $R/$O/eager.err; exit 1; }
cat $R/$O/eager.json
python3 $R/tools/rocpd_timeline.py $(ls /tmp/et/*.db /tmp/et/*/*.db 2>/dev/null | head -1) > $R/$O/timeline.json && cat $R/$O/timeline.json
