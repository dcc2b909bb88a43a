#!/bin/bash
# round 5 (n): capture tests + the captured-step probe
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_capture.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/probe_captured_step.py > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -30 $O/probe.err; exit 1; }
cat $O/probe.json
