set -o pipefail
for D in 1 2; do GNNREC_LIB=$PWD/tools/_diag/libgnnrec_diag$D.so timeout -k 10 200 python -u tools/probe_c5.py > gpurun_out/probe_diag$D.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/probe_diag$D.log; exit 1; }; echo DIAG=$D; grep "bought-by\|clicked-by" gpurun_out/probe_diag$D.log | cut -c1-200; done
