#!/bin/bash
# final-tree extras: the C5 bench line (traffic from r03e_c5) and the 2-rank gloo rehearsal of the multi-GPU bench path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --config c5 --minibatch off > gpurun_out/r03f_c5_bench_n1.json 2> gpurun_out/r03f_c5_bench_n1.err || { echo "c5 bench failed"; tail -20 gpurun_out/r03f_c5_bench_n1.err; exit 1; }
head -c 600 gpurun_out/r03f_c5_bench_n1.json; echo
GNNREC_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --users 1000000 --items 100000 --edges 50000000 --steps 3 --warmup 1 > gpurun_out/r03f_bench_gloo2.json 2> gpurun_out/r03f_bench_gloo2.err || { echo "gloo rehearsal failed"; tail -20 gpurun_out/r03f_bench_gloo2.err; exit 1; }
head -c 800 gpurun_out/r03f_bench_gloo2.json; echo
