#!/bin/bash
# round 4 (n): the multi-GPU bench path at 4 ranks (gloo, all four on the one GPU through the
# async RCCL emulation), small graph, against the committed one-GPU digest
set -o pipefail
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
GNNREC_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 4 --users 1000000 --items 100000 --edges 50000000 \
  --steps 3 --warmup 1 > $O/gloo4.json 2> $O/gloo4.err || { echo "gloo4 failed"; tail -30 $O/gloo4.err; exit 1; }
grep -o '"bitwise_vs_p1": [a-z]*' $O/gloo4.json
