#!/bin/bash
# round 6 (ac): DPP lane-group sums and readlane id broadcasts in the cosine / edge-MLP /
# cosine-backward kernels — the A/B micro benches, then the parity and capture tests
set -o pipefail
O=gpurun_out/${TAG:-r06ac}
mkdir -p $O
timeout -k 10 200 python -u tools/micro/cos_dpp_ab.py 2500 50 > $O/cos2500.json 2> $O/cos.err || { echo "cos ab failed"; tail -20 $O/cos.err; exit 1; }
cat $O/cos2500.json
timeout -k 10 200 python -u tools/micro/edge_mlp_ab.py 2500 50 > $O/mlp2500.json 2> $O/mlp.err || { echo "mlp ab failed"; tail -20 $O/mlp.err; exit 1; }
cat $O/mlp2500.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_capture.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
