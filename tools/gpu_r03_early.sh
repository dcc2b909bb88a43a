#!/bin/bash
# accumulated tiles' old partial row requested before the gather (tree) vs after (tools/_diag/prev)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py tests/test_gpu_concurrency.py -k "spmm or tile or accum or csr2 or pair or sharded or bitwise or deterministic" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_early_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_early_tests.log | head; tail -30 gpurun_out/r03_early_tests.log; exit 1; }
tail -1 gpurun_out/r03_early_tests.log
V="GNNREC_LIB=tools/_diag/prev/libgnnrec.so GNNREC_TORCH_LIB=tools/_diag/prev/libgnnrec_torch.so"
for rep in 1 2; do
  for e in "GNNREC_X=0" "$V"; do
    echo -n "C4 [$e] "
    env $e timeout -k 10 300 python bench.py --cpu-baseline off --minibatch off 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), {k: round(v,3) for k, v in r.items() if k.startswith('launch_ms') and v})" || exit 1
  done
done
bash tools/micro/c5_ab.sh "GNNREC_X=0" "$V" || exit 1
