#!/bin/bash
# Profile bench.py on the GPU box (run through gpurun from the repo root):
#   1. kernel trace + stats (per-kernel durations)
#   2. FETCH_SIZE and 3. WRITE_SIZE PMC passes on the aggregation kernels
#   4. TCC_EA0 read/write requests, all of them and those "destined for DRAM"
#   5. MFMA busy on the GEMMs
# plus <tag>_pmc_meta.json: the csrc hash the passes ran on (bench.py reports the PMC
# traffic only while the HIP sources still hash to it).
# Outputs land in gpurun_out/<tag>_*; copy the summaries to profiles/.
# Usage: bash tools/profile_round.sh <tag> [extra bench args...]
set -o pipefail
TAG=${1:-r02}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 3 --warmup 1 --cpu-baseline off --minibatch off $*"
ONE="$R/bench.py --steps 1 --warmup 0 --cpu-baseline off --minibatch off $*"

python3 -c "import sys, json; sys.path.insert(0, '$R'); import bench; \
json.dump({'csrc_sha': bench.csrc_digest(), 'bench_args': sys.argv[1:], \
'kernels': {'spmm_project': 'spmm_project_kernel', 'spmm_tile': 'spmm_csr_kernel', \
'spmm_project_mfma': 'spmm_project_mfma_kernel', 'spmm_tile2': 'spmm_csr2_kernel', 'spmm_project2': 'spmm_project2', 'spmm_pair': 'spmm_pair_mfma_kernel', \
'spmm': 'spmm_csr_kernel'}}, open('$OUT/${TAG}_pmc_meta.json', 'w'), indent=1)" $* \
  || { echo "meta failed"; exit 1; }

timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run \
  -- python3 $BENCH > "$OUT/${TAG}_trace.log" 2>&1 || { echo "trace pass failed rc=$?"; exit 1; }
echo "trace pass ok"
timeout -k 10 420 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'spmm|gemm' --output-format csv \
  -d "$OUT/${TAG}_fetch" -o run -- python3 $ONE > "$OUT/${TAG}_fetch.log" 2>&1 \
  || { echo "fetch pass failed rc=$?"; exit 1; }
echo "fetch pass ok"
timeout -k 10 420 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'spmm|gemm' --output-format csv \
  -d "$OUT/${TAG}_write" -o run -- python3 $ONE > "$OUT/${TAG}_write.log" 2>&1 \
  || { echo "write pass failed rc=$?"; exit 1; }
echo "write pass ok"
timeout -k 10 420 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum \
  TCC_EA0_WRREQ_DRAM_sum --kernel-include-regex 'spmm' --output-format csv \
  -d "$OUT/${TAG}_dram" -o run -- python3 $ONE > "$OUT/${TAG}_dram.log" 2>&1 \
  || { echo "dram pass failed rc=$?"; exit 1; }
echo "dram pass ok"
timeout -k 10 420 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE \
  --kernel-include-regex 'gemm' --output-format csv \
  -d "$OUT/${TAG}_mfma" -o run -- python3 $ONE > "$OUT/${TAG}_mfma.log" 2>&1 \
  || { echo "mfma pass failed rc=$?"; exit 1; }
echo "mfma pass ok"
