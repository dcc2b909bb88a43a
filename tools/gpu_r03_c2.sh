#!/bin/bash
# Round 3: where the C2 training step's time goes — host phases, cProfile, kernel trace.
set -o pipefail
mkdir -p gpurun_out
P=${1:-r03_c2}
timeout -k 10 200 python -u tools/probe_c2_step.py > gpurun_out/${P}_probe.txt 2>&1 || { tail -20 gpurun_out/${P}_probe.txt; exit 1; }
cat gpurun_out/${P}_probe.txt
timeout -k 10 200 python -u tools/profile_c2_host.py step > gpurun_out/${P}_cprofile.txt 2>&1 || { tail -20 gpurun_out/${P}_cprofile.txt; exit 1; }
head -60 gpurun_out/${P}_cprofile.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${P}_trace -o run -- python3 $GRAFT_REPO_ROOT/tools/probe_c2_step.py > $GRAFT_REPO_ROOT/gpurun_out/${P}_trace.log 2>&1 || { echo "trace failed"; tail $GRAFT_REPO_ROOT/gpurun_out/${P}_trace.log; exit 1; }
echo trace ok
