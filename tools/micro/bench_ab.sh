#!/bin/bash
# A/B of two libgnnrec.so builds on the C4 bench, alternating: bench_ab.sh <variant .so> [bench args]
set -o pipefail
V=${1:?variant libgnnrec.so}; shift
for rep in 1 2 3; do
  for lib in default "$V"; do
    echo -n "$lib: "
    if [ "$lib" = default ]; then
      timeout -k 10 200 python bench.py --cpu-baseline off "$@" 2>/dev/null
    else
      GNNREC_LIB=$lib timeout -k 10 200 python bench.py --cpu-baseline off "$@" 2>/dev/null
    fi | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['ms_per_step'],2), round(r.get('launch_ms_spmm_tile') or 0,3), round(r.get('launch_ms_spmm_project') or 0,3))" || exit 1
  done
done
