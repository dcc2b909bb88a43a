#!/bin/bash
# round 5 (x): device live row counts — capture / static / sampling tests, one replay
# launch by launch, the captured loop
set -o pipefail
O=gpurun_out/r05y
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_sampling.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_configs.py -k "capture or static or live or train or fold or spmm or gemm or margin or cos or head" > $O/tests.txt 2>&1 || { echo "tests failed"; tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/sq10 -o sq -- python3 $R/tools/probe_replay.py 10 20 > $R/$O/replay10.json 2> $R/$O/replay10.err || { echo "replay failed"; tail -20 $R/$O/replay10.err; exit 1; }
python3 $R/tools/rocpd_sequence.py $(ls /tmp/sq10/*.db /tmp/sq10/*/*.db 2>/dev/null | head -1) 118 > $R/$O/sequence10.txt && tail -1 $R/$O/sequence10.txt
cd $R
for K in 10 2500; do timeout -k 10 200 python3 tools/probe_captured_loop.py $K 200 || exit 1; timeout -k 10 200 python3 tools/probe_replay.py $K 50 || exit 1; done
