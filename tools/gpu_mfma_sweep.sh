set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "spmm_project or fused or c5_scale" > gpurun_out/mfma_tests.log 2>&1 || { echo "parity tests failed"; tail -40 gpurun_out/mfma_tests.log; exit 1; }
tail -1 gpurun_out/mfma_tests.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_concurrency.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/mfma_conc.log 2>&1 || { echo "concurrency tests failed"; tail -40 gpurun_out/mfma_conc.log; exit 1; }
tail -1 gpurun_out/mfma_conc.log
for U in 8 4; do GNNREC_SPM_UNROLL=$U timeout -k 10 200 python -u tools/probe_c5.py > gpurun_out/probe_c5_u$U.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/probe_c5_u$U.log; exit 1; }; echo U=$U; cut -c1-200 gpurun_out/probe_c5_u$U.log | grep -v amdgpu.ids; done
