#!/bin/bash
# round 6 (h): the item-sliced grouped cosine — bitwise tests, C3 A/B against the grouped
# form; the fused sampler's pick SQ counters
set -o pipefail
O=gpurun_out/${TAG:-r06h}
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "cos" \
  "tests/test_gpu_configs.py::test_c3_mean_nn_cosine_1024x2500_matches_oracle" \
  "tests/test_gpu_configs.py::test_c2_captured_static_steps_match_oracle" \
  -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python3 tools/micro/cos_sliced_ab.py 2500 128 50 > $O/ab128.json 2> $O/ab.err && cat $O/ab128.json || { echo "ab failed"; tail -20 $O/ab.err; exit 1; }
timeout -k 10 120 python3 tools/micro/cos_sliced_ab.py 2500 64 50 > $O/ab64.json 2>> $O/ab.err && cat $O/ab64.json || { echo "ab64 failed"; tail -20 $O/ab.err; exit 1; }
bash tools/gpu/r06g_pick_sq.sh 2>&1 | tail -12
