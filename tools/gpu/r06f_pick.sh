#!/bin/bash
# round 6 (f): the fused sampler's pick with seed byte marks and LDS-exchanged Floyd picks:
# bit-exactness, then the K = 2500 loader's kernels per grid (learned caps) and K = 10
set -o pipefail
O=gpurun_out/${TAG:-r06f}
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_sampling.py \
  "tests/test_gpu_configs.py::test_c2_csr_and_fanout_sampler_bit_exact" \
  "tests/test_gpu_configs.py::test_c2_captured_static_steps_match_oracle" \
  tests/test_gpu_capture.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
D=$R/$O/packed
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $D/trace -o lq -- python3 $R/tools/probe_loader_only.py 2500 20 auto 1 > $D.json 2> $D.err || { echo "trace failed"; tail -20 $D.err; exit 1; }
cat $D.json
python3 $R/tools/pmc_by_grid.py $D 'sb_|gather_rows_batch|cx_' | head -14
timeout -k 10 120 python3 $R/tools/probe_loader_only.py 2500 50 auto 1 > $R/$O/k2500.json 2> $R/$O/k2500.err && cat $R/$O/k2500.json
timeout -k 10 120 python3 $R/tools/probe_loader_only.py 10 100 provable 1 > $R/$O/k10.json 2> $R/$O/k10.err && cat $R/$O/k10.json
find $R/$O -name "*kernel_trace.csv" -size +20M -delete
