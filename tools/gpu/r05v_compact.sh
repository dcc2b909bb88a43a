#!/bin/bash
# round 5 (v): chained compaction scan — capture / static tests, the loader's kernel budget,
# and the captured loop
set -o pipefail
O=gpurun_out/r05v
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_parity.py -k "capture or static or compact or gemm_tn or head" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
for N in 50 150; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/lq$N -o rp -- python3 $R/tools/probe_loader_only.py 10 $N > $R/$O/loader$N.json 2> $R/$O/loader$N.err || { echo "loader $N failed"; tail -20 $R/$O/loader$N.err; exit 1; }
  cp $(ls /tmp/lq$N/*kernel_stats.csv /tmp/lq$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/loader${N}_kernel_stats.csv
done
cd $R && python3 tools/kstats_diff.py $O/loader50_kernel_stats.csv $O/loader150_kernel_stats.csv 100 > $O/loader_k10_per_batch.txt && head -8 $O/loader_k10_per_batch.txt
for K in 10 2500; do timeout -k 10 200 python3 tools/probe_captured_loop.py $K 200 || exit 1; done
