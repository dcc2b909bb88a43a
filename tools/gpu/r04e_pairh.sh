#!/bin/bash
# round 4 (e): two-phase one-table pair kernel with the self rows requested before the gathers
set -o pipefail
mkdir -p gpurun_out/r04e
O=gpurun_out/r04e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "pair" > $O/tests.log 2>&1 || { echo "pair tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in twophase pre twophase pre; do
  E="GNNREC_SPQ_PIPE=0"; [ $v = pre ] && E="GNNREC_PAIR_RAW=0"
  env $E timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_spmm_p','frac_spmm_p'))})"
done
