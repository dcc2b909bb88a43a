#!/bin/bash
# round 6 final tree (b): the small rehearsal graph's and C5's one-GPU digests (added to
# gpurun_out/r06fin/p1_digests.json), the driver's 8-GPU command rehearsed with 8 gloo ranks
# on this GPU against them, and every rank's compute share of C4 at P = 1/2/4/8
set -o pipefail
O=gpurun_out/${TAG:-r06fin}
mkdir -p $O
SMALL="--users 1000000 --items 100000 --edges 50000000"
timeout -k 10 300 python -u bench.py $SMALL --steps 3 --warmup 1 --minibatch off --cpu-baseline off \
  --record-digest $O/p1_digests.json > $O/small_n1.json 2> $O/small_n1.err || { echo "small failed"; tail -20 $O/small_n1.err; exit 1; }
echo "small ok"
timeout -k 10 400 python -u bench.py --config c5 --minibatch off --cpu-baseline off --record-digest $O/p1_digests.json \
  > $O/c5_bench_n1.json 2> $O/c5_bench_n1.err || { echo "c5 bench failed"; tail -20 $O/c5_bench_n1.err; exit 1; }
head -c 200 $O/c5_bench_n1.json; echo
GNNREC_DIST_BACKEND=gloo timeout -k 20 600 python -u bench.py --gpus 8 $SMALL --steps 3 --warmup 1 \
  --p1-digests $O/p1_digests.json > $O/gloo8.json 2> $O/gloo8.err || { echo "gloo8 failed"; tail -40 $O/gloo8.err; exit 1; }
python3 - "$O/gloo8.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print({k: c.get(k) for k in ("ranks_seen", "bitwise_vs_p1", "collective_path", "all_gather_choice")}, d["n_gpus"], d["ms_per_step"])
PY
timeout -k 10 900 python -u tools/probe_rank_work.py --config c4 --out $O/rank_compute_c4.json 1 2 4 8 \
  > $O/rank.log 2> $O/rank.err || { echo "rank probe failed"; tail -20 $O/rank.err; exit 1; }
grep '"P"' $O/rank.log | grep -v ranks | head -8
