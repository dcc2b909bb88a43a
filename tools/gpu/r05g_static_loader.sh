#!/bin/bash
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python -u tools/probe_static_loader.py > $O/loader.json 2> $O/loader.err || { echo "probe failed"; tail -30 $O/loader.err; exit 1; }
cat $O/loader.json
