#!/bin/bash
# round 5 (e): where the captured step breaks (forward / + backward / + optimizer), each
# stage only after the previous one succeeded
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
for st in fwd bwd step; do
  timeout -k 10 120 python -u tools/capture_probe.py $st > $O/probe_$st.log 2>&1 || { echo "stage $st failed"; tail -40 $O/probe_$st.log; exit 1; }
  tail -3 $O/probe_$st.log
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_capture.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
