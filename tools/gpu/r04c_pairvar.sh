#!/bin/bash
# round 4 (c): the one-table pair kernel's phase split and gather unroll (timing builds in
# tools/_diag, same soname, GNNREC_LIB): C5 pass with each, the pair launch's event time
set -o pipefail
mkdir -p gpurun_out/r04c
O=gpurun_out/r04c
for v in main spq_p1 spq_p2 spq_lu1 spq_lu3 main; do
  L=""; [ $v != main ] && L="GNNREC_LIB=$PWD/tools/_diag/libgnnrec_$v.so"
  env $L timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_','frac_'))})"
done
