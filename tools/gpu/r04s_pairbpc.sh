#!/bin/bash
# round 4 (s): how the one-table pair launch's phases scale with waves per CU — one block (8
# waves) vs two (16) per CU, gather phase alone / MFMA phase alone / whole launch (timing
# builds of a copy of the kernel with the blocks-per-CU factor as a macro, tools/_diag)
set -o pipefail
mkdir -p gpurun_out/r04s
O=gpurun_out/r04s
run() {  # name, env...
  local v=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; return 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_spmm_p','frac_spmm_p'))})"
}
for v in spq_p1_bpc2 spq_p1_bpc1 spq_p2 spq_p2_bpc1 spq_bpc1; do
  run $v GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=f32 GNNREC_LIB=$PWD/tools/_diag/libgnnrec_$v.so || exit 1
done
