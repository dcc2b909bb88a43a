#!/bin/bash
# round 6 (y): the LDS-staged edge MLP (per-edge and grouped) against the register-gather
# kernel at C3's shape, then the head tests
set -o pipefail
O=gpurun_out/${TAG:-r06y}
mkdir -p $O
timeout -k 10 120 python -u tools/micro/edge_mlp_ab.py 2500 50 > $O/ab2500.json 2> $O/ab2500.err || { echo "ab failed"; tail -20 $O/ab2500.err; exit 1; }
cat $O/ab2500.json
timeout -k 10 120 python -u tools/micro/edge_mlp_ab.py 10 200 > $O/ab10.json 2> $O/ab10.err || { echo "ab10 failed"; tail -20 $O/ab10.err; exit 1; }
cat $O/ab10.json
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "edge_mlp or predict or nn" -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
