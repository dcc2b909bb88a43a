#!/bin/bash
# pair launch's pre-projections staged at the layer start: tests, C5 A/B, C5 trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_configs.py tests/test_gpu_async.py -k "pair or c5 or side or two_ranks" -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pairearly_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_pairearly_tests.log | head; tail -30 gpurun_out/r03_pairearly_tests.log; exit 1; }
tail -1 gpurun_out/r03_pairearly_tests.log
bash tools/micro/c5_ab.sh "GNNREC_PAIR_STAGE=0" "GNNREC_PAIR_STAGE=1" || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03_pairearly_trace -o run -- python3 $R/bench.py --config c5 --steps 2 --warmup 1 --cpu-baseline off --minibatch off > $R/gpurun_out/r03_pairearly_trace.log 2>&1 || { echo "trace failed"; exit 1; }
echo trace ok
