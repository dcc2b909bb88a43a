#!/bin/bash
# round 6 (x): the loader's sampling stream at high priority vs normal, captured C2 step
set -o pipefail
O=gpurun_out/${TAG:-r06x}
mkdir -p $O
for spec in "2500 40" "10 100"; do
  set -- $spec
  timeout -k 10 400 python -u tools/probe_prefetch_priority.py $1 $2 2 > $O/k$1.json 2> $O/k$1.err || { echo "K $1 failed"; tail -20 $O/k$1.err; exit 1; }
  cat $O/k$1.json
done
