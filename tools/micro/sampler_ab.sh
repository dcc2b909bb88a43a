#!/bin/bash
# C2 sampler throughput of the current build vs a previous one (tools/_diag/prev/ holds its
# libgnnrec.so + libgnnrec_torch.so), alternating; full outputs in gpurun_out/samp_<v>_<rep>.json
set -o pipefail
for rep in 1 2; do
  for v in cur prev; do
    if [ $v = prev ]; then
      GNNREC_LIB=tools/_diag/prev/libgnnrec.so GNNREC_TORCH_LIB=tools/_diag/prev/libgnnrec_torch.so \
        timeout -k 10 300 python tools/bench_minibatch.py --batches 30 > gpurun_out/samp_${v}_$rep.json 2>/dev/null
    else
      timeout -k 10 300 python tools/bench_minibatch.py --batches 30 > gpurun_out/samp_${v}_$rep.json 2>/dev/null
    fi || exit 1
  done
done
