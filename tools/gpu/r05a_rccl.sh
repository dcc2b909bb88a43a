#!/bin/bash
# round 5 (a): RCCL on the box (nccl group of world size 1, every collective forced) and the
# self-spawning multi-rank bench (no torchrun): 2 gloo ranks on one GPU vs a fresh P=1 digest
set -o pipefail
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl.py -x -v --timeout 300 --timeout-method thread \
  > $O/rccl_tests.log 2>&1 || { echo "rccl tests failed"; tail -40 $O/rccl_tests.log; exit 1; }
tail -6 $O/rccl_tests.log
SMALL="--users 1000000 --items 100000 --edges 50000000"
timeout -k 10 300 python -u bench.py $SMALL --steps 3 --warmup 1 --minibatch off --cpu-baseline off \
  --record-digest $O/p1_digests.json > $O/p1_small.json 2> $O/p1_small.err || { echo "p1 small failed"; tail -20 $O/p1_small.err; exit 1; }
GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 $SMALL --steps 3 --warmup 1 \
  --p1-digests $O/p1_digests.json > $O/spawn2.json 2> $O/spawn2.err || { echo "spawn2 failed"; tail -30 $O/spawn2.err; exit 1; }
python -c "import json;d=json.load(open('$O/spawn2.json'));c=d['config'];print(d['n_gpus'],{k:c[k] for k in ('bitwise_vs_p1','bitwise_vs_p1_src','rank_edges','rank_compute_ms','collective_path')})"
if WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 timeout -k 10 120 python bench.py --gpus 2 $SMALL > $O/mismatch.out 2> $O/mismatch.err; then
  echo "mismatch run exited 0 (should fail)"; exit 1
fi
echo "mismatch refused: $(tail -1 $O/mismatch.err)"
