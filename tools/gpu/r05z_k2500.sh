#!/bin/bash
# round 5 (z): K = 2500 — one replay launch by launch, and the static loader's per-batch
# kernel budget (differenced stats)
set -o pipefail
O=gpurun_out/r05z
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sq -o sq -- python3 $R/tools/probe_replay.py 2500 10 > $R/$O/replay.json 2> $R/$O/replay.err || { echo "replay failed"; tail -20 $R/$O/replay.err; exit 1; }
python3 $R/tools/rocpd_sequence.py $(ls /tmp/sq/*.db /tmp/sq/*/*.db 2>/dev/null | head -1) 110 > $R/$O/sequence2500.txt && tail -1 $R/$O/sequence2500.txt
for N in 20 60; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lq$N -o rp -- python3 $R/tools/probe_loader_only.py 2500 $N > $R/$O/loader$N.json 2> $R/$O/loader$N.err || { echo "loader $N failed"; tail -20 $R/$O/loader$N.err; exit 1; }
  cp $(ls /tmp/lq$N/*kernel_stats.csv /tmp/lq$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/loader${N}_kernel_stats.csv
done
cd $R && python3 tools/kstats_diff.py $O/loader20_kernel_stats.csv $O/loader60_kernel_stats.csv 40 > $O/loader_k2500_per_batch.txt && head -25 $O/loader_k2500_per_batch.txt
