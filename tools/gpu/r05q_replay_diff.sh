#!/bin/bash
# round 5 (q): the K = 10 replay's kernel budget exactly: kernel stats at N = 50 and N = 150
# replays, differenced (tools/kstats_diff.py)
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 50 150; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rq$N -o rp -- python3 $R/tools/probe_replay.py 10 $N > $R/$O/replay$N.json 2> $R/$O/replay$N.err || { echo "replay $N failed"; tail -20 $R/$O/replay$N.err; exit 1; }
  cat $R/$O/replay$N.json
  cp $(ls /tmp/rq$N/*kernel_stats.csv /tmp/rq$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/replay${N}_kernel_stats.csv
done
cd $R && python3 tools/kstats_diff.py $O/replay50_kernel_stats.csv $O/replay150_kernel_stats.csv 100 > $O/replay_k10_per_step.txt && cat $O/replay_k10_per_step.txt
