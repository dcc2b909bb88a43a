#!/bin/bash
# round 6 (m): the K = 2500 step's kernel budgets, per step, apples to apples: the eager loop
# without the sampling thread (kernels serialised, no contention) and the captured replay at
# learned capacities (the bench's form)
set -o pipefail
O=gpurun_out/${TAG:-r06m}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 20 60; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/e$N -o e -- python3 $R/tools/probe_eager_step.py 2500 $N 0 > $R/$O/eager$N.json 2> $R/$O/eager$N.err || { echo "eager $N failed"; tail -20 $R/$O/eager$N.err; exit 1; }
  cp $(ls /tmp/e$N/*kernel_stats.csv /tmp/e$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/eager${N}.csv
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r$N -o r -- python3 $R/tools/probe_replay.py 2500 $N auto > $R/$O/replay$N.json 2> $R/$O/replay$N.err || { echo "replay $N failed"; tail -20 $R/$O/replay$N.err; exit 1; }
  cp $(ls /tmp/r$N/*kernel_stats.csv /tmp/r$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/replay${N}.csv
done
cd $R && python3 tools/kstats_diff.py $O/eager20.csv $O/eager60.csv 60 > $O/eager_budget.txt && python3 tools/kstats_diff.py $O/replay20.csv $O/replay60.csv 60 > $O/replay_budget.txt && head -1 $O/eager_budget.txt $O/replay_budget.txt
cat $O/eager60.json $O/replay60.json
