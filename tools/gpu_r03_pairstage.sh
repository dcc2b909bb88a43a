#!/bin/bash
# one-rank trees on the side stream + pair pre-projections queued ahead: tests, C5 and C4 A/B
set -o pipefail
mkdir -p gpurun_out
true || timeout -k 10 700 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_configs.py tests/test_gpu_async.py tests/test_gpu_parity.py -k "pair or c5 or c4 or side or two_ranks or sharded or pass" -q --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/r03_pairstage_tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/r03_pairstage_tests.log | head; tail -30 gpurun_out/r03_pairstage_tests.log; exit 1; }
tail -1 gpurun_out/r03_pairstage_tests.log
bash tools/micro/c5_ab.sh "GNNREC_TREE_SIDE=0 GNNREC_PAIR_STAGE=0" "GNNREC_TREE_SIDE=1 GNNREC_PAIR_STAGE=0" "GNNREC_TREE_SIDE=1 GNNREC_PAIR_STAGE=1" || exit 1
for rep in 1 2; do
  for e in "GNNREC_TREE_SIDE=0" "GNNREC_TREE_SIDE=1"; do
    echo -n "C4 [$e] "
    env $e timeout -k 10 300 python bench.py --cpu-baseline off --minibatch off 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],2))" || exit 1
  done
done
