#!/bin/bash
# round 4 (i): is the fp32 GEMM's output store its floor?  1M x 256 x 128 (one, sage forms)
# with the normal store, non-temporal stores, and no store (timing build); MFMA busy and
# WRITE_SIZE per variant from separate PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04i
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in main gemm_nt gemm_nost; do
    L=""; [ $v != main ] && L="GNNREC_LIB=$R/tools/_diag/libgnnrec_$v.so"
    for form in one sage; do
      echo "$v $(env $L timeout -k 10 60 python3 $R/tools/micro/gemm_one.py 1000000 256 128 20 $form)" || exit 1
    done
  done
done
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for v in main gemm_nt gemm_nost; do
  L=""; [ $v != main ] && L="$R/tools/_diag/libgnnrec_$v.so"
  for P in "$P1" "WRITE_SIZE"; do
    tag=$v-$(echo $P | cut -c1-8)
    GNNREC_LIB=${L:-$R/gnn-recsys_amd/gnnrec/libgnnrec.so} timeout -s KILL 60 rocprofv3 --pmc $P --kernel-include-regex gemm --output-format csv -d $O/pmc_$tag -o run -- python3 $R/tools/micro/gemm_one.py 1000000 256 128 5 one > $O/pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/pmc_$tag.log; exit 1; }
    echo "pmc $tag ok"
  done
done
