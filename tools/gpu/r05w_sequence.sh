#!/bin/bash
# round 5 (w): one captured replay launch by launch (K = 10 and 2500)
set -o pipefail
O=gpurun_out/r05w
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for K in 10 2500; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sq$K -o sq -- python3 $R/tools/probe_replay.py $K 20 > $R/$O/replay$K.json 2> $R/$O/replay$K.err || { echo "replay $K failed"; tail -20 $R/$O/replay$K.err; exit 1; }
  python3 $R/tools/rocpd_sequence.py $(ls /tmp/sq$K/*.db /tmp/sq$K/*/*.db 2>/dev/null | head -1) 118 > $R/$O/sequence$K.txt && tail -1 $R/$O/sequence$K.txt
done
