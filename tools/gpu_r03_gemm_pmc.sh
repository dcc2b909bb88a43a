#!/bin/bash
# Round 3: where the short-K fp32 GEMM's cycles go (instruction mix per MFMA, co-execution).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for form in one sage; do
  timeout -k 10 60 python3 $R/tools/micro/gemm_one.py 1000000 256 128 20 $form || exit 1
done
P1="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_WAIT_INST_ANY"
i=0
for form in one sage; do
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $P --kernel-include-regex gemm --output-format csv -d $R/gpurun_out/r03_gemm_pmc$i -o run -- python3 $R/tools/micro/gemm_one.py 1000000 256 128 5 $form > $R/gpurun_out/r03_gemm_pmc$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/r03_gemm_pmc$i.log; exit 1; }
    echo "pass $i ($form) ok"
  done
done
