#!/bin/bash
# round 5 (b): the fused sampler (gnnrec_sample_blocks) and the grouped cosine head — their
# tests, the C2 bit-exact config test, a same-box sampler A/B against the per-layer path, and
# the minibatch rooflines (sampler, cosine, edge MLP)
set -o pipefail
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampling.py tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "sampl or gather_rows_batch or stamp or c2 or loader or prefetch or cos" > $O/tests.log 2>&1 || { echo "tests failed"; tail -60 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
timeout -k 10 300 python -u tools/sampler_ab.py 50 > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail -30 $O/ab.err; exit 1; }
cat $O/ab.json
timeout -k 10 300 python -u tools/minibatch_roofline.py > $O/mb_roof.json 2> $O/mb_roof.err || { echo "mb roofline failed"; tail -20 $O/mb_roof.err; exit 1; }
cat $O/mb_roof.json
