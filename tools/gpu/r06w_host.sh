#!/bin/bash
# round 6 (w): the captured C2 loop's host split (tools/probe_host_split.py) at K = 2500 / 10
set -o pipefail
O=gpurun_out/${TAG:-r06w}
mkdir -p $O
for K in 2500 10; do
  timeout -k 10 300 python -u tools/probe_host_split.py $K 60 > $O/host$K.json 2> $O/host$K.err || { echo "K $K failed"; tail -20 $O/host$K.err; exit 1; }
  cat $O/host$K.json
done
