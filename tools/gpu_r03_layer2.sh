#!/bin/bash
# layer node incl. fc_preagg: tests, then kernel traces of C2 and C3 with GNNREC_TRAIN_LAYER 0/1
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_parity.py -k "train or fused or layer or autograd or edge_loader or golden" -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_layer_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_layer_tests.log | head; tail -30 gpurun_out/r03_layer_tests.log; exit 1; }
tail -1 gpurun_out/r03_layer_tests.log
cd /tmp && export TMPDIR=/tmp
for l in 0 1; do
  GNNREC_TRAIN_LAYER=$l GNNREC_COS_PAIR=$l timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_l${l}_c2 -o run -- python3 $R/tools/probe_c2_step.py 10 0 > $R/gpurun_out/r03_l${l}_c2.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03_l${l}_c2.log; exit 1; }
  GNNREC_TRAIN_LAYER=$l GNNREC_COS_PAIR=$l timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r03_l${l}_c3 -o run -- python3 $R/tools/probe_c2_step.py 2500 0 128 mean_nn > $R/gpurun_out/r03_l${l}_c3.log 2>&1 || { echo "trace failed"; tail $R/gpurun_out/r03_l${l}_c3.log; exit 1; }
done
echo traces ok
