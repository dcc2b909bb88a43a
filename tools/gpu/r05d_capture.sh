#!/bin/bash
# round 5 (d): static-shape blocks / batch head and the captured training step
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_capture.py tests/test_gpu_sampling.py -m gpu -x -v \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -80 $O/tests.log; exit 1; }
tail -5 $O/tests.log
