#!/bin/bash
# round 6 (o): the K = 10 captured step's parts — the static loader's per-batch kernel budget
# and the replay's (kernel stats at two run lengths, differenced)
set -o pipefail
O=gpurun_out/${TAG:-r06o}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 40 120; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/l$N -o l -- python3 $R/tools/probe_loader_only.py 10 $N provable 1 > $R/$O/loader$N.json 2> $R/$O/loader$N.err || { echo "loader $N failed"; tail -20 $R/$O/loader$N.err; exit 1; }
  cp $(ls /tmp/l$N/*kernel_stats.csv /tmp/l$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/loader${N}.csv
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r$N -o r -- python3 $R/tools/probe_replay.py 10 $N provable > $R/$O/replay$N.json 2> $R/$O/replay$N.err || { echo "replay $N failed"; tail -20 $R/$O/replay$N.err; exit 1; }
  cp $(ls /tmp/r$N/*kernel_stats.csv /tmp/r$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/replay${N}.csv
done
cd $R && python3 tools/kstats_diff.py $O/loader40.csv $O/loader120.csv 80 > $O/loader_budget.txt && python3 tools/kstats_diff.py $O/replay40.csv $O/replay120.csv 80 > $O/replay_budget.txt && head -30 $O/loader_budget.txt && head -1 $O/replay_budget.txt
cat $O/loader120.json $O/replay120.json
