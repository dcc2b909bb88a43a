#!/bin/bash
# training layer as one autograd node (GNNREC_TRAIN_LAYER): tests, then C2 / C3 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_parity.py -k "train or fused or layer or autograd or edge_loader or golden" -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_layer_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_layer_tests.log | head; tail -30 gpurun_out/r03_layer_tests.log; exit 1; }
tail -1 gpurun_out/r03_layer_tests.log
for rep in 1 2; do
  for l in 0 1; do
    echo "LAYER=$l $(GNNREC_TRAIN_LAYER=$l timeout -k 10 200 python -u tools/probe_c2_step.py 10 2 2>/dev/null | tail -1)"
    echo "LAYER=$l $(GNNREC_TRAIN_LAYER=$l timeout -k 10 200 python -u tools/probe_c2_step.py 10 0 2>/dev/null | tail -1)"
  done
done
for l in 0 1; do
  echo "LAYER=$l $(GNNREC_TRAIN_LAYER=$l timeout -k 10 200 python -u tools/probe_c2_step.py 2500 2 128 mean_nn 2>/dev/null | tail -1)"
done
