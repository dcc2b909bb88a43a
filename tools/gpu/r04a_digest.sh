#!/bin/bash
# round 4 (a): the multi-GPU bench's self-check rehearsed on one GPU — P=1 digests (small
# graph and full C4), the 2-rank gloo rehearsal compared with them (bitwise_vs_p1 true), the
# same with one rank's output perturbed (false); the minibatch kernels' rooflines + rocprof
set -o pipefail
mkdir -p gpurun_out/r04a
O=gpurun_out/r04a
export TMPDIR=/tmp
SMALL="--users 1000000 --items 100000 --edges 50000000"
timeout -k 10 300 python -u bench.py $SMALL --steps 3 --warmup 1 --minibatch off --cpu-baseline off \
  --record-digest $O/p1_digests.json > $O/p1_small.json 2> $O/p1_small.err || { echo "p1 small failed"; tail -20 $O/p1_small.err; exit 1; }
head -c 400 $O/p1_small.json; echo
GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 $SMALL --steps 3 --warmup 1 \
  --p1-digests $O/p1_digests.json > $O/gloo2.json 2> $O/gloo2.err || { echo "gloo2 failed"; tail -30 $O/gloo2.err; exit 1; }
python -c "import json;d=json.load(open('$O/gloo2.json'))['config'];print({k:d[k] for k in ('output_digest','bitwise_vs_p1','bitwise_vs_p1_src','rank_edges','rank_compute_ms','ms_per_step_replicated_output')})"
GNNREC_BENCH_PERTURB_RANK=1 GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 $SMALL --steps 3 --warmup 1 \
  --p1-digests $O/p1_digests.json > $O/gloo2_perturbed.json 2> $O/gloo2_perturbed.err || { echo "gloo2 perturbed failed"; tail -30 $O/gloo2_perturbed.err; exit 1; }
python -c "import json;d=json.load(open('$O/gloo2_perturbed.json'))['config'];print({k:d[k] for k in ('output_digest','bitwise_vs_p1')})"
timeout -k 10 300 python -u tools/minibatch_roofline.py > $O/mb_roof.json 2> $O/mb_roof.err || { echo "mb roofline failed"; tail -20 $O/mb_roof.err; exit 1; }
cat $O/mb_roof.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mb -o mb -- python3 tools/minibatch_roofline.py > $O/mb_roof_prof.json 2> $O/mb_roof_prof.err || { echo "mb rocprof failed"; tail -20 $O/mb_roof_prof.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
  --record-digest $O/p1_digests.json > $O/p1_c4.json 2> $O/p1_c4.err || { echo "p1 c4 failed"; tail -20 $O/p1_c4.err; exit 1; }
head -c 600 $O/p1_c4.json; echo
