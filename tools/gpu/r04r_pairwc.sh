#!/bin/bash
# round 4 (r): the fp32 one-table pair launch's weight-stream depth — B operands per
# double-buffered chunk (GNNREC_SPQ_WC 8 / 16 / 32, timing builds in tools/_diag): the MFMA
# phase alone and the whole launch, C5 pass with the raw pair (GNNREC_PAIR_RAW=1)
set -o pipefail
mkdir -p gpurun_out/r04r
O=gpurun_out/r04r
run() {  # name, env...
  local v=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; return 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_spmm_p','frac_spmm_p'))})"
}
for v in spq_p2wc8 spq_p2 spq_p2wc32 spq_wc8 spq_wc32; do
  run $v GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=f32 GNNREC_LIB=$PWD/tools/_diag/libgnnrec_$v.so || exit 1
done
run main GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=f32 || exit 1
