#!/bin/bash
# round 5 (u): the static loader's per-batch kernel budget at K = 10 (stats at N = 50 and 150
# batches, differenced)
set -o pipefail
O=gpurun_out/r05u
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for N in 50 150; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lq$N -o rp -- python3 $R/tools/probe_loader_only.py 10 $N > $R/$O/loader$N.json 2> $R/$O/loader$N.err || { echo "loader $N failed"; tail -20 $R/$O/loader$N.err; exit 1; }
  cp $(ls /tmp/lq$N/*kernel_stats.csv /tmp/lq$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/loader${N}_kernel_stats.csv
done
cd $R && python3 tools/kstats_diff.py $O/loader50_kernel_stats.csv $O/loader150_kernel_stats.csv 100 > $O/loader_k10_per_batch.txt && cat $O/loader_k10_per_batch.txt
