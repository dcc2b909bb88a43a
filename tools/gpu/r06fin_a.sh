#!/bin/bash
# round 6 final tree (a): the GPU suite, smoke, and the default bench line with the C4
# one-GPU digest recorded into a copy of the committed digest file
set -o pipefail
O=gpurun_out/${TAG:-r06fin}
mkdir -p $O
cp profiles/p1_output_digests.json $O/p1_digests.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py --record-digest $O/p1_digests.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
