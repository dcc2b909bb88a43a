set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gputest.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gputest.log; exit 1; }
tail -3 gpurun_out/gputest.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || { echo "bench failed"; tail -20 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
GNNREC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --users 1000000 --items 100000 --edges 50000000 --steps 3 --warmup 1 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { echo "gloo rehearsal failed"; tail -20 gpurun_out/bench_gloo2.err; exit 1; }
cat gpurun_out/bench_gloo2.json
bash tools/profile_round.sh r02_c4 || exit 1
