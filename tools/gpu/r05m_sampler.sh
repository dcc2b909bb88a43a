#!/bin/bash
# round 5 (m): block data gathered inside the fused sampler op — sampling / capture tests,
# the minibatch rooflines, the captured-step probe
set -o pipefail
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_capture.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python -u tools/minibatch_roofline.py > $O/mb_roof.json 2> $O/mb_roof.err || { echo "mb roofline failed"; tail -20 $O/mb_roof.err; exit 1; }
python -c "import json; d=json.load(open('$O/mb_roof.json')); print(json.dumps(d['sampler']))"
timeout -k 10 400 python -u tools/probe_captured_step.py > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -30 $O/probe.err; exit 1; }
cat $O/probe.json
