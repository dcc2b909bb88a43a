#!/bin/bash
# round 5 (ac): the eager K = 2500 C2 step's kernel budget, loader included (stats at
# N = 20 and 60 steps, differenced)
set -o pipefail
O=gpurun_out/r05ac
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 20 60; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/eq$N -o rp -- python3 $R/tools/probe_eager_step.py 2500 $N > $R/$O/eager$N.json 2> $R/$O/eager$N.err || { echo "eager $N failed"; tail -20 $R/$O/eager$N.err; exit 1; }
  cat $R/$O/eager$N.json
  cp $(ls /tmp/eq$N/*kernel_stats.csv /tmp/eq$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/eager${N}_kernel_stats.csv
done
cd $R && python3 tools/kstats_diff.py $O/eager20_kernel_stats.csv $O/eager60_kernel_stats.csv 40 > $O/eager_k2500_per_step.txt && head -40 $O/eager_k2500_per_step.txt
