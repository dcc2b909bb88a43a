#!/bin/bash
# round 6 (d): seed bitmaps in the fused sampler's pick + finalize's loads hoisted:
# bit-exactness, then the K = 2500 loader trace (learned capacities, packed) + PMC per grid
set -o pipefail
O=gpurun_out/${TAG:-r06d}
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sampling.py \
  "tests/test_gpu_configs.py::test_c2_csr_and_fanout_sampler_bit_exact" \
  "tests/test_gpu_configs.py::test_c2_captured_static_steps_match_oracle" \
  tests/test_gpu_capture.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
K='sb_|gather_rows_batch|cx_'
D=$R/$O/packed
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o lq -- python3 $R/tools/probe_loader_only.py 2500 20 auto 1 > $D.json 2> $D.err || { echo "trace failed"; tail -20 $D.err; exit 1; }
cat $D.json
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $D/fetch -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 auto 1 > $D/fetch.json 2> $D/fetch.err || { echo "fetch pass failed"; tail -20 $D/fetch.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $D/write -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 auto 1 > $D/write.json 2> $D/write.err || { echo "write pass failed"; tail -20 $D/write.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" --output-format csv -d $D/hit -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 auto 1 > $D/hit.json 2> $D/hit.err || { echo "hit pass failed"; tail -20 $D/hit.err; exit 1; }
python3 $R/tools/pmc_by_grid.py $D "$K" > $R/$O/summary_packed.md
cat $R/$O/summary_packed.md
timeout -k 10 120 python3 $R/tools/probe_loader_only.py 10 100 provable 1 > $R/$O/k10.json 2> $R/$O/k10.err && cat $R/$O/k10.json
find $R/$O -name "*kernel_trace.csv" -size +20M -delete
