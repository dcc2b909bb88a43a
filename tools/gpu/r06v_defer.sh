#!/bin/bash
# round 6 (v): the static loader's overflow flag read one batch late — sampling / capture
# GPU tests, then the captured K = 2500 / K = 10 steps (probe_captured_ab: lazy vs gathered
# block data, the same process)
set -o pipefail
O=gpurun_out/${TAG:-r06v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sampling.py tests/test_gpu_capture.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/probe_captured_ab.py 2500 40 2 > $O/k2500.json 2> $O/k2500.err || { echo "k2500 failed"; tail -20 $O/k2500.err; exit 1; }
cat $O/k2500.json
timeout -k 10 300 python -u tools/probe_captured_ab.py 10 100 2 > $O/k10.json 2> $O/k10.err || { echo "k10 failed"; tail -20 $O/k10.err; exit 1; }
cat $O/k10.json
