for b in 4 6 8 32; do
  echo "== blocks_per_cu=$b"
  GNNREC_SPMM_BLOCKS_PER_CU=$b timeout -k 10 200 python tools/bench_kernels.py --only spmm --zipf 0 2>&1 | grep -A3 "zipf0\"" | grep -E "spmm|\"ms\"" 
  GNNREC_SPMM_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --cpu-baseline off --steps 4 2>&1 | grep metric | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('pass ms', r['ms_per_step'], 'value', r['value']/1e9)"
done
