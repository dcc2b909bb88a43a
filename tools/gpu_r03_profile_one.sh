#!/bin/bash
# one config's round record: its bench line, then tools/profile_round.sh (kernel trace + PMC)
#   bash tools/gpu_r03_profile_one.sh <tag, e.g. r03b_c4> [bench args, e.g. --config c5]
set -o pipefail
T=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py "$@" > gpurun_out/${T}_bench_n1.json 2> gpurun_out/${T}_bench_n1.err || { echo "bench failed"; tail -20 gpurun_out/${T}_bench_n1.err; exit 1; }
cat gpurun_out/${T}_bench_n1.json
bash tools/profile_round.sh ${T} "$@" || exit 1
