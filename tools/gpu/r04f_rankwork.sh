#!/bin/bash
# round 4 (f): every rank's compute share of the C4 and C5 passes at P = 1/2/4/8 on the
# current sources (tools/probe_rank_work.py), with the projected scaling curve
set -o pipefail
mkdir -p gpurun_out/r04f
O=gpurun_out/r04f
timeout -k 10 900 python -u tools/probe_rank_work.py --config c4 --out $O/rank_compute_c4.json 1 2 4 8 \
  > $O/c4.log 2> $O/c4.err || { echo "c4 probe failed"; tail -20 $O/c4.err; exit 1; }
grep '"P"' $O/c4.log | grep -v ranks | head -8
