#!/bin/bash
# round 4 (t): the one-table pair launch with three blocks per CU (24 waves; 80 VGPRs per lane
# forced, spilling), gather lockstep unroll 2 / 1, B chunk 16 / 8 — whole launch, C5 pass
set -o pipefail
mkdir -p gpurun_out/r04t
O=gpurun_out/r04t
run() {  # name, env...
  local v=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; return 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_spmm_p','frac_spmm_p'))})"
}
for v in ${VARIANTS:-spq_b3lu2 spq_b3lu1 spq_b3lu1wc8}; do
  run $v GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=f32 GNNREC_LIB=$PWD/tools/_diag/libgnnrec_$v.so || exit 1
done
run main GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=f32 || exit 1
