#!/bin/bash
# round 4 final tree (z2): the C4 bench line as the driver runs it, and the one-GPU output
# digests of C4 and of the small rehearsal graph, added to a copy of the committed digest file
# (gpurun_out/r04z/p1_digests.json -> profiles/p1_output_digests.json afterwards)
set -o pipefail
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
if [ -f profiles/p1_output_digests.json ]; then cp profiles/p1_output_digests.json $O/p1_digests.json; fi
timeout -k 10 600 python -u bench.py --record-digest $O/p1_digests.json > $O/c4_bench_n1.json 2> $O/c4_bench_n1.err || { echo "c4 bench failed"; tail -20 $O/c4_bench_n1.err; exit 1; }
head -c 600 $O/c4_bench_n1.json; echo
timeout -k 10 300 python -u bench.py --users 1000000 --items 100000 --edges 50000000 --steps 3 --warmup 1 \
  --minibatch off --cpu-baseline off --record-digest $O/p1_digests.json > $O/small_n1.json 2> $O/small_n1.err || { echo "small failed"; exit 1; }
echo "small ok"
