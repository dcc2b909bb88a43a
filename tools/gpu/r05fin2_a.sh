#!/bin/bash
# round 5 final tree, second pass (a): the whole GPU suite, smoke, the default bench line (C4 digest
# recorded) and the small rehearsal graph's one-GPU digest, added to a copy of the committed
# digest file (gpurun_out/r05fin2/p1_digests.json -> profiles/p1_output_digests.json)
set -o pipefail
O=gpurun_out/r05fin2
mkdir -p $O
if [ -f profiles/p1_output_digests.json ]; then cp profiles/p1_output_digests.json $O/p1_digests.json; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --record-digest $O/p1_digests.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-600
timeout -k 10 300 python -u bench.py --users 1000000 --items 100000 --edges 50000000 --steps 3 --warmup 1 \
  --minibatch off --cpu-baseline off --record-digest $O/p1_digests.json > $O/small_n1.json 2> $O/small_n1.err || { echo "small failed"; tail -20 $O/small_n1.err; exit 1; }
echo "small ok"
