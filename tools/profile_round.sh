#!/bin/bash
# Profile bench.py on the GPU box (run through gpurun from the repo root):
#   1. kernel trace + stats (per-kernel durations)
#   2. FETCH_SIZE and 3. WRITE_SIZE PMC passes on the aggregation kernels
# Outputs land in gpurun_out/<tag>_*; copy the summaries to profiles/.
# Usage: bash tools/profile_round.sh <tag> [extra bench args...]
set -o pipefail
TAG=${1:-r01}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 3 --warmup 1 --cpu-baseline off $*"

timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run \
  -- python3 $BENCH > "$OUT/${TAG}_trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace pass ok"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'spmm|gemm' --output-format csv \
  -d "$OUT/${TAG}_fetch" -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-baseline off $* \
  > "$OUT/${TAG}_fetch.log" 2>&1 || { echo "fetch pass failed rc=$?"; exit 1; }
echo "fetch pass ok"
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'spmm|gemm' --output-format csv \
  -d "$OUT/${TAG}_write" -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-baseline off $* \
  > "$OUT/${TAG}_write.log" 2>&1 || { echo "write pass failed rc=$?"; exit 1; }
echo "write pass ok"
timeout -k 10 420 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE \
  --kernel-include-regex 'gemm' --output-format csv \
  -d "$OUT/${TAG}_mfma" -o run -- python3 $R/bench.py --steps 1 --warmup 0 --cpu-baseline off $* \
  > "$OUT/${TAG}_mfma.log" 2>&1 || { echo "mfma pass failed rc=$?"; exit 1; }
echo "mfma pass ok"
