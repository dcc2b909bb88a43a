#!/bin/bash
# Round 3: the compile-time GEMM epilogue — parity, A/B against the runtime-flag epilogue, VALU count.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_parity.py -k "gemm or project or golden" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/r03_gemm_ab.log 2>&1 || { tail -30 $R/gpurun_out/r03_gemm_ab.log; exit 1; }
tail -1 $R/gpurun_out/r03_gemm_ab.log
for rep in 1 2 3; do
  for form in one sage; do
    for f in 1 0; do
      echo -n "FAST_EPI=$f "; GNNREC_GEMM_FAST_EPI=$f timeout -k 10 60 python3 $R/tools/micro/gemm_one.py 1000000 256 128 20 $form || exit 1
    done
  done
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
i=10
for form in one sage; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $P1 --kernel-include-regex gemm --output-format csv -d $R/gpurun_out/r03_gemm_pmc$i -o run -- python3 $R/tools/micro/gemm_one.py 1000000 256 128 5 $form > $R/gpurun_out/r03_gemm_pmc$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
  echo "pass $i ($form) ok"
done
