#!/bin/bash
# round 4 final tree (z2): the C4 bench line as the driver runs it, the one-GPU output digests
# of C4 and of the small rehearsal graph (profiles/p1_output_digests.json), then the C4
# rocprof record (kernel trace + PMC passes, tools/profile_round.sh)
set -o pipefail
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
timeout -k 10 600 python -u bench.py --record-digest $O/p1_digests.json > $O/c4_bench_n1.json 2> $O/c4_bench_n1.err || { echo "c4 bench failed"; tail -20 $O/c4_bench_n1.err; exit 1; }
head -c 400 $O/c4_bench_n1.json; echo
timeout -k 10 300 python -u bench.py --users 1000000 --items 100000 --edges 50000000 --steps 3 --warmup 1 \
  --minibatch off --cpu-baseline off --record-digest $O/p1_digests.json > $O/small_n1.json 2> $O/small_n1.err || { echo "small failed"; exit 1; }
timeout -k 10 1200 bash tools/profile_round.sh r04z_c4 || exit 1
