#!/bin/bash
# round 4 final tree (z4): the 2-rank gloo rehearsal of the multi-GPU bench path against the
# committed one-GPU digests (profiles/p1_output_digests.json), once as is and once with one
# bit of rank 1's output flipped; then the minibatch kernels' rooflines under rocprofv3
set -o pipefail
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
SMALL="--users 1000000 --items 100000 --edges 50000000"
GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 $SMALL --steps 3 --warmup 1 \
  > $O/gloo2.json 2> $O/gloo2.err || { echo "gloo2 failed"; tail -30 $O/gloo2.err; exit 1; }
GNNREC_BENCH_PERTURB_RANK=1 GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 $SMALL --steps 3 --warmup 1 \
  > $O/gloo2_perturbed.json 2> $O/gloo2_perturbed.err || { echo "perturbed failed"; exit 1; }
grep -o '"bitwise_vs_p1": [a-z]*' $O/gloo2.json $O/gloo2_perturbed.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_mb -o mb -- python3 $GRAFT_REPO_ROOT/tools/minibatch_roofline.py \
  > $GRAFT_REPO_ROOT/$O/mb_roof_prof.json 2> $GRAFT_REPO_ROOT/$O/mb_roof_prof.err || { echo "mb rocprof failed"; exit 1; }
echo "mb ok"
