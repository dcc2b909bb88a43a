#!/bin/bash
# (round 5 (k), reused for the final round-6 tree): the minibatch kernels (C2 sampler, C3 grouped cosine, C3 edge MLP): kernel
# trace + separate PMC passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss), summarised here
set -o pipefail
O=${O:-gpurun_out/r06fmb}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
K='sb_|gather_rows_batch|sddmm_cos|edge_mlp'
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o mb -- python3 $R/tools/minibatch_roofline.py 20 > $R/$O/trace.json 2> $R/$O/trace.err || { echo "trace failed"; tail -20 $R/$O/trace.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $R/$O/fetch -o mb -- python3 $R/tools/minibatch_roofline.py 20 > $R/$O/fetch.json 2> $R/$O/fetch.err || { echo "fetch pass failed"; tail -20 $R/$O/fetch.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $R/$O/write -o mb -- python3 $R/tools/minibatch_roofline.py 20 > $R/$O/write.json 2> $R/$O/write.err || { echo "write pass failed"; tail -20 $R/$O/write.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" --output-format csv -d $R/$O/hit -o mb -- python3 $R/tools/minibatch_roofline.py 20 > $R/$O/hit.json 2> $R/$O/hit.err || { echo "hit pass failed"; tail -20 $R/$O/hit.err; exit 1; }
python3 $R/tools/pmc_summary.py $R/$O > $R/$O/summary.md || { echo "summary failed"; exit 1; }
cat $R/$O/summary.md
find $R/$O -name "*kernel_trace.csv" -delete
