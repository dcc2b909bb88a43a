#!/bin/bash
# C2 GPU-time cuts: row-queue ticket cap, 64x64 weight-gradient tile, 16-deep GEMM at N=64
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sampling.py tests/test_gpu_torch_ops.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_c2e_tests.log 2>&1 || { tail -40 gpurun_out/r03_c2e_tests.log; exit 1; }
tail -1 gpurun_out/r03_c2e_tests.log
for e in 0 1; do
  for shape in "257000 64 64" "204000 128 64" "100000 64 64"; do
    echo "BK16_N64=$e $shape: $(GNNREC_GEMM_BK16_N64=$e timeout -k 10 60 python tools/micro/gemm_one.py $shape 20 2>/dev/null | tail -1)"
  done
done
for rep in 1 2; do
  for nw in 0 2; do
    timeout -k 10 120 python -u tools/probe_c2_step.py 10 $nw 2>/dev/null | tail -1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_c2e_nw0 -o run -- python3 $R/tools/probe_c2_step.py 10 0 > $R/gpurun_out/r03_c2e_nw0.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03_c2e_nw0.log; exit 1; }
tail -1 $R/gpurun_out/r03_c2e_nw0.log
