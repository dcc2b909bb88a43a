#!/bin/bash
# round 5 final tree, second pass (b): the C5 bench line and its one-GPU digest, then the C4 rocprof
# record (kernel trace + PMC passes, tools/profile_round.sh) on the final kernels
set -o pipefail
O=gpurun_out/r05fin2
mkdir -p $O
if [ -f profiles/p1_output_digests.json ]; then cp profiles/p1_output_digests.json $O/p1_digests_c5.json; fi
timeout -k 10 400 python -u bench.py --config c5 --minibatch off --cpu-baseline off --record-digest $O/p1_digests_c5.json \
  > $O/c5_bench_n1.json 2> $O/c5_bench_n1.err || { echo "c5 bench failed"; tail -20 $O/c5_bench_n1.err; exit 1; }
head -c 400 $O/c5_bench_n1.json; echo
timeout -k 10 900 bash tools/profile_round.sh r05fin2_c4 || exit 1
