#!/bin/bash
# A/B of a GEMM tuning knob (an env var read once by libgnnrec.so), alternating 1 / 0:
#   bash tools/micro/gemm_ab.sh GNNREC_GEMM_BK16
set -o pipefail
VAR=${1:?env var to toggle}
for shape in "1000000 256" "2000000 256" "1000000 128" "2000000 128"; do
  for rep in 1 2; do
    for w in 1 0; do
      echo -n "$VAR=$w "
      env "$VAR=$w" timeout -k 10 60 python tools/micro/gemm_one.py $shape 128 20 || exit 1
    done
  done
done
