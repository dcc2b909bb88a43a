#!/bin/bash
# round 4 (j2): phase split of the bf16x3 pair launch (gather alone / MFMA alone) and its
# B-chunk depth — timing builds in tools/_diag (GNNREC_LIB), C5 pass with the raw pair
set -o pipefail
mkdir -p gpurun_out/r04j
O=gpurun_out/r04j
run() {  # name, env...
  local v=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; return 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_spmm_p','frac_spmm_p'))})"
}
for v in spq_p1 spq_p2 spq_bc1 spq_bc4; do
  run ${v}_bf3 GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=bf16x3 GNNREC_LIB=$PWD/tools/_diag/libgnnrec_$v.so || exit 1
done
run spq_p2_f32 GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=f32 GNNREC_LIB=$PWD/tools/_diag/libgnnrec_spq_p2.so || exit 1
