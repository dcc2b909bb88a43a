#!/bin/bash
# round 5 (ae): per-step kernel budget of the eager K = 2500 C2 loop on the final sources
# (kernel stats at 20 and 60 steps, differenced by tools/kstats_diff.py)
set -o pipefail
O=gpurun_out/${OUT:-r05ae}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 20 60; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k$N -o k$N -- python3 $R/tools/probe_eager_step.py 2500 $N > $R/$O/eager$N.json 2> $R/$O/eager$N.err || { echo "trace $N failed"; tail -20 $R/$O/eager$N.err; exit 1; }
  cp $(ls /tmp/k$N/*kernel_stats.csv /tmp/k$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/k$N.csv
done
python3 $R/tools/kstats_diff.py $R/$O/k20.csv $R/$O/k60.csv 40 > $R/$O/budget.txt && head -45 $R/$O/budget.txt
