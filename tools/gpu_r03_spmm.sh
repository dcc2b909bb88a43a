#!/bin/bash
# low-degree spmm (minibatch block relation): row-queue ticket size / static schedule
set -o pipefail
for shape in "100000 10 100000 64" "100000 10 257000 64" "20000 10 257000 64" "1000000 10 100000 64"; do
  timeout -k 10 60 python tools/micro/spmm_one.py $shape 20 mean 2>/dev/null | tail -1 || exit 1
  GNNREC_ROWQ=0 timeout -k 10 60 python tools/micro/spmm_one.py $shape 20 mean 2>/dev/null | sed 's/^/static /' | tail -1 || exit 1
  for c in 1 4 16 51; do
    GNNREC_RQ_CHUNK=$c timeout -k 10 60 python tools/micro/spmm_one.py $shape 20 mean 2>/dev/null | sed "s/^/chunk$c /" | tail -1 || exit 1
  done
done
