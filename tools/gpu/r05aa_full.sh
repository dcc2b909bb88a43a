#!/bin/bash
# round 5 (aa): the whole GPU suite, smoke and the default bench line on the current tree
set -o pipefail
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-3000
