#!/bin/bash
# round 5 (s): fewer launches in the captured step — the training tests that cover the
# changed paths, then the K = 10 replay budget (differenced kernel stats) and the step
set -o pipefail
O=gpurun_out/r05s
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py -k "capture or fold or gemm_tn or train or margin or cos" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
for N in 50 150; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rq$N -o rp -- python3 $R/tools/probe_replay.py 10 $N > $R/$O/replay$N.json 2> $R/$O/replay$N.err || { echo "replay $N failed"; tail -20 $R/$O/replay$N.err; exit 1; }
  cp $(ls /tmp/rq$N/*kernel_stats.csv /tmp/rq$N/*/*kernel_stats.csv 2>/dev/null | head -1) $R/$O/replay${N}_kernel_stats.csv
done
cd $R && python3 tools/kstats_diff.py $O/replay50_kernel_stats.csv $O/replay150_kernel_stats.csv 100 > $O/replay_k10_per_step.txt && head -30 $O/replay_k10_per_step.txt
timeout -k 10 300 python3 -u tools/probe_captured_step.py 10 --captured-only > $O/step10.json 2> $O/step10.err || { echo "step probe failed"; tail -20 $O/step10.err; exit 1; }
cat $O/step10.json
