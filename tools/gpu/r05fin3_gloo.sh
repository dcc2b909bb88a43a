#!/bin/bash
# round 5 final tree (third pass): the 2-rank gloo rehearsal of the multi-GPU bench path (ranks
# sharing the one GPU) against the committed one-GPU digests of these sources
set -o pipefail
O=gpurun_out/r05fin3
mkdir -p $O
GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --users 1000000 --items 100000 --edges 50000000 \
  --steps 3 --warmup 1 > $O/gloo2.json 2> $O/gloo2.err || { echo "gloo2 failed"; tail -30 $O/gloo2.err; exit 1; }
grep -o '"bitwise_vs_p1": [a-z]*' $O/gloo2.json
