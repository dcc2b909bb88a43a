#!/bin/bash
# round 5 (o): the captured step's replay alone, kernel stats
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for K in 10 2500; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp$K -o rp -- python3 $R/tools/probe_replay.py $K 50 > $R/$O/replay$K.json 2> $R/$O/replay$K.err || { echo "replay $K failed"; tail -20 $R/$O/replay$K.err; exit 1; }
  cat $R/$O/replay$K.json
  cp $(ls /tmp/rp$K/*kernel_stats.csv /tmp/rp$K/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/replay${K}_kernel_stats.csv
done
