#!/bin/bash
# round 6 (u): K = 2500 on the lazy-data tree — the static loader's per-batch kernel budget
# (stats at 20 and 60 batches, differenced) and the captured loop's timeline (overlap of the
# loader's stream with the replays)
set -o pipefail
O=gpurun_out/${TAG:-r06u}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 20 60; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/l$N -o l -- python3 $R/tools/probe_loader_only.py 2500 $N auto 1 > $R/$O/loader$N.json 2> $R/$O/loader$N.err || { echo "loader $N failed"; tail -20 $R/$O/loader$N.err; exit 1; }
  cp $(ls /tmp/l$N/*kernel_stats.csv /tmp/l$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/loader${N}.csv
done
cd $R && python3 tools/kstats_diff.py $O/loader20.csv $O/loader60.csv 40 > $O/loader_budget.txt && head -30 $O/loader_budget.txt && cat $O/loader60.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/tl -o tl -- python3 $R/tools/probe_captured_loop.py 2500 100 0 2 auto > $R/$O/loop.json 2> $R/$O/loop.err || { echo "loop failed"; tail -20 $R/$O/loop.err; exit 1; }
cat $R/$O/loop.json
python3 $R/tools/rocpd_timeline.py $(ls /tmp/tl/*.db /tmp/tl/*/*.db 2>/dev/null | head -1) > $R/$O/timeline.json && cat $R/$O/timeline.json
