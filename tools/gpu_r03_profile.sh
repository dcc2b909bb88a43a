#!/bin/bash
# Round 3 record on one MI355X: the C4 and C5 bench lines, then rocprofv3 kernel traces and
# PMC passes of both (tools/profile_round.sh), all under gpurun_out/.
#   bash tools/gpu_r03_profile.sh <tag prefix, e.g. r03a>
set -o pipefail
P=${1:-r03a}
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/${P}_c4_bench.json 2> gpurun_out/${P}_c4_bench.err || { echo "C4 bench failed"; tail -20 gpurun_out/${P}_c4_bench.err; exit 1; }
cat gpurun_out/${P}_c4_bench.json
timeout -k 10 300 python -u bench.py --config c5 --cpu-baseline off > gpurun_out/${P}_c5_bench.json 2> gpurun_out/${P}_c5_bench.err || { echo "C5 bench failed"; tail -20 gpurun_out/${P}_c5_bench.err; exit 1; }
cat gpurun_out/${P}_c5_bench.json
bash tools/profile_round.sh ${P}_c4 || exit 1
bash tools/profile_round.sh ${P}_c5 --config c5 || exit 1
