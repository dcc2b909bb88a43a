#!/bin/bash
# kernel trace only (no PMC) of one bench config: timeline of the last pass
#   bash tools/gpu_r03_trace.sh <tag> [bench args]
set -o pipefail
T=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/${T}_trace -o run \
  -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-baseline off --minibatch off "$@" > $R/gpurun_out/${T}_trace.log 2>&1 || { echo "trace failed"; tail -20 $R/gpurun_out/${T}_trace.log; exit 1; }
f=$(find $R/gpurun_out/${T}_trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline.py $f --last-ms 160 > $R/gpurun_out/${T}_timeline.txt && tail -1 $R/gpurun_out/${T}_timeline.txt
