#!/bin/bash
# round 6 (b): the K = 2500 static loader's kernels per dispatch grid (step 0 / step 1 of the
# fused sampler apart): kernel trace + FETCH / WRITE / L2-hit PMC passes
set -o pipefail
O=gpurun_out/${TAG:-r06b}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
K='sb_|gather_rows_batch|cx_'
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/$O/trace -o lq -- python3 $R/tools/probe_loader_only.py 2500 20 > $R/$O/trace.json 2> $R/$O/trace.err || { echo "trace failed"; tail -20 $R/$O/trace.err; exit 1; }
cat $R/$O/trace.json
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $R/$O/fetch -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 > $R/$O/fetch.json 2> $R/$O/fetch.err || { echo "fetch pass failed"; tail -20 $R/$O/fetch.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $R/$O/write -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 > $R/$O/write.json 2> $R/$O/write.err || { echo "write pass failed"; tail -20 $R/$O/write.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" --output-format csv -d $R/$O/hit -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 > $R/$O/hit.json 2> $R/$O/hit.err || { echo "hit pass failed"; tail -20 $R/$O/hit.err; exit 1; }
python3 $R/tools/pmc_by_grid.py $R/$O "$K" > $R/$O/summary.md || { echo "summary failed"; exit 1; }
cat $R/$O/summary.md
find $R/$O -name "*kernel_trace.csv" -size +20M -delete
