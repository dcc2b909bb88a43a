#!/bin/bash
# round 4 final tree (z3): the C5 bench line + its one-GPU digest, and its rocprof record
set -o pipefail
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
if [ -f profiles/p1_output_digests.json ]; then cp profiles/p1_output_digests.json $O/p1_digests_c5.json; fi
timeout -k 10 400 python -u bench.py --config c5 --minibatch off --cpu-baseline off --record-digest $O/p1_digests_c5.json \
  > $O/c5_bench_n1.json 2> $O/c5_bench_n1.err || { echo "c5 bench failed"; tail -20 $O/c5_bench_n1.err; exit 1; }
head -c 600 $O/c5_bench_n1.json; echo
timeout -k 10 900 bash tools/profile_round.sh r04z_c5 --config c5 || exit 1
