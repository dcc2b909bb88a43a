#!/bin/bash
# round 5 (l): capture / sampling tests (learned static capacities, overflow), then the
# minibatch PMC job (r05k) and the captured-step probe
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_capture.py tests/test_gpu_sampling.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/gpu/r05k_mb_pmc.sh || exit 1
timeout -k 10 400 python -u tools/probe_captured_step.py > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -30 $O/probe.err; exit 1; }
cat $O/probe.json
