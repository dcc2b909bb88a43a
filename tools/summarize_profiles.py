"""Summarise committed rocprofv3 outputs (profiles/<tag>_*.csv) into roofline numbers.

    python tools/summarize_profiles.py r01_c4

gfx950 corrections (MI355X_MICROARCH.md §HBM, §rocprofv3): FETCH_SIZE counts half the
bytes of wide coalesced reads (x2); WRITE_SIZE is exact; both in KB.  GRBM_GUI_ACTIVE is
summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES sums the busy cycles of all 1024 SIMDs,
so MFMA-busy = busy / (GRBM_GUI_ACTIVE / 8 * 1024).  TCC_EA0_RDREQ_DRAM counts every
memory-side read request, Infinity-Cache hits included (it equals TCC_EA0_RDREQ on these
kernels): no gfx950 counter in ROCm 7.2 separates DRAM from MALL traffic.
"""
import csv
import os
import sys
from collections import defaultdict

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles")


def short(name):
    return name.split("(anonymous namespace)::", 1)[-1].split("(")[0]


def main(tag):
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(ROOT, tag + "_kernel_stats.csv")))}
    print("| kernel | calls | avg ms |")
    print("|---|---|---|")
    for n, r in stats.items():
        if "gnnrec" in n:
            print(f"| `{short(n)}` | {r['Calls']} | {float(r['AverageNs']) / 1e6:.3f} |")
    per = defaultdict(lambda: defaultdict(float))
    for kind, scale in (("fetch", 2.0), ("write", 1.0), ("mfma", 1.0), ("dram", 1.0)):
        p = os.path.join(ROOT, f"{tag}_pmc_{kind}.csv")
        if not os.path.exists(p):
            continue
        for r in csv.DictReader(open(p)):
            key = (r["Dispatch_Id"], short(r["Kernel_Name"]), r["Grid_Size"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"]) * (scale if kind == "fetch" else 1)
    print()
    print("| dispatch | kernel | grid | HBM read GB (FETCH x2) | HBM write GB | EA read req "
          "(of them 'DRAM') | MFMA busy |")
    print("|---|---|---|---|---|---|---|")
    for key in sorted(per, key=lambda k: int(k[0])):
        v = per[key]
        rd = v.get("FETCH_SIZE", 0) * 1024 / 1e9
        wr = v.get("WRITE_SIZE", 0) * 1024 / 1e9
        mb = ""
        if "SQ_VALU_MFMA_BUSY_CYCLES" in v and v.get("GRBM_GUI_ACTIVE"):
            mb = f"{100 * v['SQ_VALU_MFMA_BUSY_CYCLES'] / (v['GRBM_GUI_ACTIVE'] / 8 * 1024):.0f} %"
        rq = ""
        if "TCC_EA0_RDREQ_sum" in v:
            rq = (f"{v['TCC_EA0_RDREQ_sum'] / 1e9:.3f} G ({v['TCC_EA0_RDREQ_DRAM_sum'] / 1e9:.3f} G)")
        print(f"| {key[0]} | `{key[1]}` | {key[2]} | {rd:.1f} | {wr:.2f} | {rq} | {mb} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01_c4")
