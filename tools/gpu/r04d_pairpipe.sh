#!/bin/bash
# round 4 (d): the software-pipelined one-table pair kernel — parity, then C5 A/B against the
# two-phase form (GNNREC_SPQ_PIPE=0), the pre-projected launch (GNNREC_PAIR_RAW=0) and the
# pipelined form with a 2-deep lockstep (tools/_diag/libgnnrec_spq_plu2.so)
set -o pipefail
mkdir -p gpurun_out/r04d
O=gpurun_out/r04d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "pair or project2" > $O/tests.log 2>&1 || { echo "pair tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in pipe twophase pre plu2; do
  E=""
  case $v in twophase) E="GNNREC_SPQ_PIPE=0";; pre) E="GNNREC_PAIR_RAW=0";; plu2) E="GNNREC_LIB=$PWD/tools/_diag/libgnnrec_spq_plu2.so";; esac
  env $E timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_','frac_'))})"
done
