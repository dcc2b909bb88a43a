#!/bin/bash
# round 4 (j): the one-table pair launch with its projections as six bf16 MFMA products of
# three-way split operands (bf16x3) against the fp32-MFMA form and the pre-projected launch:
# pair tests, then the C5 pass per variant (alternating), then the bf16x3 phase split and
# B-chunk depth (timing builds in tools/_diag, GNNREC_LIB)
set -o pipefail
mkdir -p gpurun_out/r04j
O=gpurun_out/r04j
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "pair" > $O/tests.log 2>&1 || { echo "pair tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # name, env...
  local v=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --config c5 --steps 5 --warmup 2 --minibatch off --cpu-baseline off \
    > $O/c5_$v.json 2> $O/c5_$v.err || { echo "c5 $v failed"; tail -20 $O/c5_$v.err; return 1; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],2), {k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k.startswith(('launch_ms_spmm_p','frac_spmm_p'))})"
}
for rep in 1 2; do
  run bf3_$rep GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=bf16x3 || exit 1
  run f32_$rep GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=f32 || exit 1
  run pre_$rep GNNREC_PAIR_RAW=0 || exit 1
done
for v in spq_p1 spq_p2 spq_bc1 spq_bc4; do
  run $v GNNREC_PAIR_RAW=1 GNNREC_PAIR_MFMA=bf16x3 GNNREC_LIB=$PWD/tools/_diag/libgnnrec_$v.so || exit 1
done
