#!/bin/bash
# fast GEMM epilogue with wave-local syncs (tools/_diag/ews, GEMM_EPI_WAVE_SYNC=1) vs block barriers (tree)
set -o pipefail
mkdir -p gpurun_out
V="GNNREC_LIB=tools/_diag/ews/libgnnrec.so GNNREC_TORCH_LIB=tools/_diag/ews/libgnnrec_torch.so"
env $V timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "gemm or project or golden or sage or train or c5" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_ews_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_ews_tests.log | head; tail -30 gpurun_out/r03_ews_tests.log; exit 1; }
tail -1 gpurun_out/r03_ews_tests.log
for rep in 1 2 3; do
  for shape in "1000000 256 128 20 one" "1000000 256 128 20 sage" "1000000 128 128 20 one"; do
    echo "tree $(timeout -k 10 60 python3 tools/micro/gemm_one.py $shape)" || exit 1
    echo "ews  $(env $V timeout -k 10 60 python3 tools/micro/gemm_one.py $shape)" || exit 1
  done
done
bash tools/micro/c5_ab.sh "GNNREC_X=0" "$V" || exit 1
