#!/bin/bash
# round 5 (c): after the knob pruning — the whole GPU suite + smoke, then the minibatch
# rooflines (sampler, grouped cosine, edge MLP) and a rocprofv3 kernel trace of them
set -o pipefail
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -60 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/minibatch_roofline.py > $O/mb_roof.json 2> $O/mb_roof.err || { echo "mb roofline failed"; tail -20 $O/mb_roof.err; exit 1; }
cat $O/mb_roof.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_mb -o mb -- python3 $GRAFT_REPO_ROOT/tools/minibatch_roofline.py \
  > $GRAFT_REPO_ROOT/$O/mb_roof_prof.json 2> $GRAFT_REPO_ROOT/$O/mb_roof_prof.err || { echo "mb rocprof failed"; exit 1; }
echo "mb prof ok"
