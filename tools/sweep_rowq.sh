#!/bin/bash
# Row-queue tuning sweep on the C4 bench (run through gpurun from the repo root):
#   bash tools/sweep_rowq.sh  -> gpurun_out/sweep_rowq.log (one line per setting)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sweep_rowq.log
mkdir -p "$R/gpurun_out"; : > "$OUT"
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-baseline off \
    > "$R/gpurun_out/sweep_$tag.log" 2>&1 || { echo "$tag failed rc=$?" >> "$OUT"; exit 1; }
  python3 - "$tag" "$R/gpurun_out/sweep_$tag.log" >> "$OUT" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[1], round(d["ms_per_step"], 2), "fused", round(r["launch_ms"], 3),
      "tile", round(r["other_kernels"]["spmm_tile"]["launch_ms"], 3), flush=True)
PY
}
run default X=0
run chunk1 GNNREC_RQ_CHUNK=1
run chunk4 GNNREC_RQ_CHUNK=4
run fused2 GNNREC_RQ_CHUNK_FUSED=2
run fused8 GNNREC_RQ_CHUNK_FUSED=8
run bpc6 GNNREC_SPMM_BLOCKS_PER_CU=6
cat "$OUT"
