#!/bin/bash
# round 5 (d): static-shape blocks / batch head, the captured training step, the minibatch
# rooflines
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "grouped or cosine" -m gpu -x -v \
  --timeout 120 --timeout-method thread > $O/cos_tests.log 2>&1 || { echo "cos tests failed"; tail -60 $O/cos_tests.log; exit 1; }
tail -2 $O/cos_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_capture.py tests/test_gpu_sampling.py -m gpu -x -v \
  --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -80 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 python -u tools/probe_captured_step.py > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -30 $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 300 python -u tools/minibatch_roofline.py > $O/mb_roof.json 2> $O/mb_roof.err || { echo "mb roofline failed"; tail -20 $O/mb_roof.err; exit 1; }
cat $O/mb_roof.json
