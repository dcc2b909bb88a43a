#!/bin/bash
# weight-gradient GEMM (64 x 64 tile, 64-row steps) + scans: tests, micro shapes, C2 probe + trace
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "scan or relabel or gemm_tn or backward" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_wg_tests.log 2>&1 || { tail -40 gpurun_out/r03_wg_tests.log; exit 1; }
tail -1 gpurun_out/r03_wg_tests.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_torch_ops.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_wg_tests2.log 2>&1 || { tail -40 gpurun_out/r03_wg_tests2.log; exit 1; }
tail -1 gpurun_out/r03_wg_tests2.log
for shape in "1024 64 64" "10000 64 64" "100000 64 64" "204000 64 64" "400000 64 64" "1000000 128 128"; do
  timeout -k 10 60 python tools/micro/gemm_tn_one.py $shape 2>/dev/null | tail -1 || exit 1
done
for rep in 1 2; do
  for nw in 0 2; do
    timeout -k 10 120 python -u tools/probe_c2_step.py 10 $nw 2>/dev/null | tail -1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_wg_nw0 -o run -- python3 $R/tools/probe_c2_step.py 10 0 > $R/gpurun_out/r03_wg_nw0.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03_wg_nw0.log; exit 1; }
tail -1 $R/gpurun_out/r03_wg_nw0.log
