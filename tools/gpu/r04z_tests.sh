#!/bin/bash
# round 4 final tree (z1): the whole GPU suite and smoke, as the driver runs them
set -o pipefail
mkdir -p gpurun_out/r04z
O=gpurun_out/r04z
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/gputest.log 2>&1 || { echo "gpu tests failed"; tail -40 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
