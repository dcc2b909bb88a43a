#!/bin/bash
# the driver's round-end checks on one MI355X: the whole GPU suite, then the C4 bench line
#   bash tools/gpu_full.sh <tag>
set -o pipefail
P=${1:-full}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${P}_gputest.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|error" gpurun_out/${P}_gputest.log | tail -20; tail -30 gpurun_out/${P}_gputest.log; exit 1; }
tail -3 gpurun_out/${P}_gputest.log
timeout -k 10 300 python -u bench.py > gpurun_out/${P}_bench_n1.json 2> gpurun_out/${P}_bench_n1.err || { echo "bench failed"; tail -20 gpurun_out/${P}_bench_n1.err; exit 1; }
cat gpurun_out/${P}_bench_n1.json
