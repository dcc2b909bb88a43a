#!/bin/bash
# round 6 (j): the captured K = 2500 step's replay kernel budget on the current sources
# (kernel stats of two replay counts, differenced: per replay)
set -o pipefail
O=gpurun_out/${TAG:-r06j}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 20 60; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rq$N -o rp -- python3 $R/tools/probe_replay.py 2500 $N > $R/$O/replay$N.json 2> $R/$O/replay$N.err || { echo "replay $N failed"; tail -20 $R/$O/replay$N.err; exit 1; }
  cp $(ls /tmp/rq$N/*kernel_stats.csv /tmp/rq$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/replay${N}_kernel_stats.csv
done
cd $R && python3 tools/kstats_diff.py $O/replay20_kernel_stats.csv $O/replay60_kernel_stats.csv 40 > $O/replay_k2500_per_step.txt && head -45 $O/replay_k2500_per_step.txt
cat $O/replay60.json
