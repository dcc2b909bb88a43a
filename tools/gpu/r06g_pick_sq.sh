#!/bin/bash
# round 6 (g): what bounds the fused sampler's pick at K = 2500 — SQ counters (wave cycles,
# waits, instruction mix) per dispatch grid
set -o pipefail
O=gpurun_out/${TAG:-r06g}
mkdir -p $O
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/$O/counters.txt 2>&1 || true
grep -oE "SQ_[A-Z_0-9]+" $R/$O/counters.txt | sort -u > $R/$O/sq_names.txt || true
D=$R/$O/sq
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex "sb_pick|sb_finalize|gather_rows_batch" --output-format csv -d $D -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 auto 1 > $D.json 2> $D.err || { echo "sq pass failed"; tail -20 $D.err; exit 1; }
D2=$R/$O/sq2
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES --kernel-include-regex "sb_pick|sb_finalize|gather_rows_batch" --output-format csv -d $D2 -o lq -- python3 $R/tools/probe_loader_only.py 2500 10 auto 1 > $D2.json 2> $D2.err || { echo "sq2 pass failed"; tail -5 $D2.err; }
python3 - "$R/$O" <<'PY'
import csv, glob, sys, collections, re
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("gnnrec::(anonymous namespace)::", ""))
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or "0"
        acc[(k, int(g))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key in sorted(acc):
    c = acc[key]
    print(key, {n: round(sum(v) / len(v)) for n, v in sorted(c.items())})
PY
