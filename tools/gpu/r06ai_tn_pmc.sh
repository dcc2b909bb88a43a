#!/bin/bash
# round 6 (ai): the d = 64 weight gradient (K = 1M rows, 64 x 64) under PMC passes — fetch /
# write bytes, L2 hits, wave-state counters
set -o pipefail
O=gpurun_out/${TAG:-r06ai}
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
K='gemm_tn'
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d $R/$O/fetch -o t -- python3 $R/tools/micro/gemm_tn_one.py 1000000 64 64 10 > /dev/null 2>&1 || { echo "fetch failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d $R/$O/write -o t -- python3 $R/tools/micro/gemm_tn_one.py 1000000 64 64 10 > /dev/null 2>&1 || { echo "write failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$K" --output-format csv -d $R/$O/hit -o t -- python3 $R/tools/micro/gemm_tn_one.py 1000000 64 64 10 > /dev/null 2>&1 || { echo "hit failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-include-regex "$K" --output-format csv -d $R/$O/sq -o t -- python3 $R/tools/micro/gemm_tn_one.py 1000000 64 64 10 > /dev/null 2>&1 || { echo "sq failed"; exit 1; }
cd $R && python3 - $O <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "partial" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, round(sum(v) / len(v), 1))
PY
