#!/bin/bash
# C2 training step (tools/probe_c2_step.py) of the current build vs tools/_diag/prev/, alternating
set -o pipefail
for rep in 1 2 3; do
  for v in cur prev; do
    echo -n "$v: "
    if [ $v = prev ]; then
      GNNREC_LIB=tools/_diag/prev/libgnnrec.so GNNREC_TORCH_LIB=tools/_diag/prev/libgnnrec_torch.so \
        timeout -k 10 300 python tools/probe_c2_step.py 2>/dev/null | grep wall
    else
      timeout -k 10 300 python tools/probe_c2_step.py 2>/dev/null | grep wall
    fi || exit 1
  done
done
