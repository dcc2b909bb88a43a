#!/bin/bash
# round 5 final tree, fifth pass (after the grouped backward's id and partial prefetch):
# the GPU suite, smoke, the default bench line (C4 digest recorded),
# the small rehearsal graph's and C5's one-GPU digests, added to a copy of the committed digest
# file (gpurun_out/r05fin5/p1_digests.json -> profiles/p1_output_digests.json)
set -o pipefail
O=gpurun_out/r05fin5
mkdir -p $O
cp profiles/p1_output_digests.json $O/p1_digests.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --record-digest $O/p1_digests.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
timeout -k 10 300 python -u bench.py --users 1000000 --items 100000 --edges 50000000 --steps 3 --warmup 1 \
  --minibatch off --cpu-baseline off --record-digest $O/p1_digests.json > $O/small_n1.json 2> $O/small_n1.err || { echo "small failed"; tail -20 $O/small_n1.err; exit 1; }
echo "small ok"
timeout -k 10 400 python -u bench.py --config c5 --minibatch off --cpu-baseline off --record-digest $O/p1_digests.json \
  > $O/c5_bench_n1.json 2> $O/c5_bench_n1.err || { echo "c5 bench failed"; tail -20 $O/c5_bench_n1.err; exit 1; }
head -c 300 $O/c5_bench_n1.json; echo
GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --users 1000000 --items 100000 --edges 50000000 \
  --steps 3 --warmup 1 --p1-digests $O/p1_digests.json > $O/gloo2.json 2> $O/gloo2.err || { echo "gloo2 failed"; tail -30 $O/gloo2.err; exit 1; }
grep -o '"bitwise_vs_p1": [a-z]*' $O/gloo2.json
