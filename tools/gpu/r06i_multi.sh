#!/bin/bash
# round 6 (i): the multi-GPU readiness — the small graph's one-GPU digest, then the exact
# command the driver runs at 8 GPUs (bench.py --gpus 8, self-spawned ranks) rehearsed with 8
# gloo ranks on this one GPU (all-gather form chosen at run time, both forms' replays in the
# diagnostics, bitwise_vs_p1), then every rank's compute share of C4 at P = 1/2/4/8
set -o pipefail
O=gpurun_out/${TAG:-r06i}
mkdir -p $O
cp profiles/p1_output_digests.json $O/p1_digests.json
SMALL="--users 1000000 --items 100000 --edges 50000000"
timeout -k 10 300 python -u bench.py $SMALL --steps 3 --warmup 1 --minibatch off --cpu-baseline off \
  --record-digest $O/p1_digests.json > $O/small_n1.json 2> $O/small_n1.err || { echo "small n1 failed"; tail -20 $O/small_n1.err; exit 1; }
echo "small n1 ok"
GNNREC_DIST_BACKEND=gloo timeout -k 20 600 python -u bench.py --gpus 8 $SMALL --steps 3 --warmup 1 \
  --p1-digests $O/p1_digests.json > $O/gloo8.json 2> $O/gloo8.err || { echo "gloo8 failed"; tail -40 $O/gloo8.err; exit 1; }
python3 - "$O/gloo8.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print({k: c.get(k) for k in ("ranks_seen", "bitwise_vs_p1", "collective_path", "all_gather_choice",
                              "comm_ms", "comm_ms_by_all_gather_mode", "rank_compute_ms")}, d["n_gpus"], d["ms_per_step"])
PY
timeout -k 10 900 python -u tools/probe_rank_work.py --config c4 --out $O/rank_compute_c4.json 1 2 4 8 \
  > $O/rank.log 2> $O/rank.err || { echo "rank probe failed"; tail -20 $O/rank.err; exit 1; }
grep '"P"' $O/rank.log | grep -v ranks | head -8
