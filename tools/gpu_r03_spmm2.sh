#!/bin/bash
# transposed-gather shapes of the K = 2500 step: row queue vs static, d = 64, weighted sum
set -o pipefail
for shape in "1000000 2 1000000 64" "1000000 3 120000 64" "300000 3 1000000 64" "100000 30 1000000 64"; do
  echo "queue  $(timeout -k 10 60 python tools/micro/spmm_one.py $shape 20 sum 1 2>/dev/null | tail -1)"
  echo "static $(GNNREC_ROWQ=0 timeout -k 10 60 python tools/micro/spmm_one.py $shape 20 sum 1 2>/dev/null | tail -1)"
done
