#!/bin/bash
# round 5 (p): host cost of the static loader (cProfile) and the captured loop's queue wait
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
for K in 10 2500; do
  timeout -k 10 300 python3 -u tools/probe_loader_host.py $K 200 > $O/host$K.txt 2> $O/host$K.err || { echo "probe $K failed"; tail -20 $O/host$K.err; exit 1; }
  head -1 $O/host$K.txt; tail -1 $O/host$K.txt
done
