#!/bin/bash
# A/B of a libgnnrec.so variant on the short-K GEMM shapes, alternating: gemm_lib_ab.sh <variant .so>
set -o pipefail
V=${1:?variant libgnnrec.so}
for shape in "1000000 256" "2000000 256" "1000000 128"; do
  for rep in 1 2 3; do
    echo -n "default "; timeout -k 10 60 python tools/micro/gemm_one.py $shape 128 20 || exit 1
    echo -n "variant "; GNNREC_LIB=$V timeout -k 10 60 python tools/micro/gemm_one.py $shape 128 20 || exit 1
  done
done
