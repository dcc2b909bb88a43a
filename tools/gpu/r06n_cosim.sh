#!/bin/bash
# round 6 (n): the item-major grouped cosine — bitwise tests, C3 A/B against the grouped form
set -o pipefail
O=gpurun_out/${TAG:-r06n}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "cos" \
  "tests/test_gpu_configs.py::test_c3_mean_nn_cosine_1024x2500_matches_oracle" \
  -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for D in 128 64; do
  timeout -k 10 120 python3 tools/micro/cos_im_ab.py 2500 $D 50 > $O/ab$D.json 2>> $O/ab.err && cat $O/ab$D.json || { echo "ab $D failed"; tail -20 $O/ab.err; exit 1; }
done
timeout -k 10 120 python3 tools/micro/cos_im_ab.py 10 64 50 > $O/ab64_k10.json 2>> $O/ab.err && cat $O/ab64_k10.json
