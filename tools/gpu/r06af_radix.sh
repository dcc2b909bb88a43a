#!/bin/bash
# round 6 (af): the radix scatter writing each tile in output order from LDS — the sort
# micro bench against the previous scatter (tools/_diag/libgnnrec_oldsort.so), then the
# CSR / sampler / capture / cosine tests
set -o pipefail
O=gpurun_out/${TAG:-r06af}
mkdir -p $O
for spec in "2561024 100000" "1000000 1100000" "50000000 1000000"; do
  set -- $spec
  for lib in new old; do
    if [ $lib = old ]; then export GNNREC_LIB=tools/_diag/libgnnrec_oldsort.so; else unset GNNREC_LIB; fi
    echo -n "$lib: "
    timeout -k 10 120 python -u tools/micro/radix_one.py $1 $2 30 2>> $O/radix.err || { echo "radix $lib failed"; tail -20 $O/radix.err; exit 1; }
  done
done | tee $O/radix.txt
unset GNNREC_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_csr.py tests/test_gpu_sampling.py tests/test_gpu_capture.py tests/test_gpu_parity.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
