#!/bin/bash
# round 4 (b): the one-table pair kernel (gnnrec_spmm_pair_f32) — parity tests, then C5
# alternating A/B against the pre-projected pair launch (GNNREC_PAIR_RAW=0)
set -o pipefail
mkdir -p gpurun_out/r04b
O=gpurun_out/r04b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "pair or project2" > $O/tests.log 2>&1 || { echo "pair tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  for raw in 1 0; do
    GNNREC_PAIR_RAW=$raw timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
      > $O/c5_raw${raw}_$i.json 2> $O/c5_raw${raw}_$i.err || { echo "c5 raw=$raw failed"; tail -20 $O/c5_raw${raw}_$i.err; exit 1; }
    python -c "import json;d=json.load(open('$O/c5_raw${raw}_$i.json'));r=d['roofline'];print('raw=$raw', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_','frac_'))})"
  done
done
