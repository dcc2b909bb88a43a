set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "gemm or project or golden or model" > gpurun_out/gemm_tests.log 2>&1 || { echo "gemm tests failed"; tail -40 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
for S in 3 2; do GNNREC_GEMM_STAGES=$S timeout -k 10 200 python -u tools/bench_gemm_k.py > gpurun_out/gemm_k_s$S.json 2>&1 || { echo "bench failed"; tail -20 gpurun_out/gemm_k_s$S.json; exit 1; }; echo S=$S; python -c "
import json,sys; d=json.load(open('gpurun_out/gemm_k_s$S.json'.replace('.json','.json')) if False else None" 2>/dev/null; grep -v amdgpu gpurun_out/gemm_k_s$S.json | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print({k:(round(v['TFs'],1), round(v.get('TFs_relu_l2',0),1), round(v['ms'],3)) for k,v in d.items() if isinstance(v,dict)})"; done
