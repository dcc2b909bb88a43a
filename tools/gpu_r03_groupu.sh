#!/bin/bash
# group kernel neighbours in flight: U = 16 (tree) vs 12 (tools/_diag/u12) vs 8 (tools/_diag/prev)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "spmm or group or backward or grad" -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_gu_tests.log 2>&1 || { tail -30 gpurun_out/r03_gu_tests.log; exit 1; }
tail -1 gpurun_out/r03_gu_tests.log
run() {  # variant, command...
  local v=$1; shift
  if [ $v = 16 ]; then "$@"; else GNNREC_LIB=tools/_diag/$v/libgnnrec.so GNNREC_TORCH_LIB=tools/_diag/$v/libgnnrec_torch.so "$@"; fi
}
for rep in 1 2; do
  for v in 16 u12 prev; do
    for shape in "630000 10 100000 64 20 mean" "100000 63 630000 64 20 sum 1" "1000000 2 100000 64 20 sum 1" "100000 10 1000000 64 20 mean"; do
      echo "U=$v $(run $v timeout -k 10 60 python tools/micro/spmm_one.py $shape 2>/dev/null | tail -1)" || exit 1
    done
  done
done
for rep in 1 2; do
  for v in 16 u12 prev; do
    echo "U=$v K2500 $(run $v timeout -k 10 200 python -u tools/probe_c2_step.py 2500 2 2>/dev/null | tail -1 | cut -c1-160)" || exit 1
    echo "U=$v K10 $(run $v timeout -k 10 200 python -u tools/probe_c2_step.py 10 2 2>/dev/null | tail -1 | cut -c1-160)" || exit 1
  done
done
