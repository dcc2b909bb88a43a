"""Per-kernel averages of a rocprofv3 kernel trace and its PMC passes (FETCH_SIZE, WRITE_SIZE,
TCC hit / miss), as a markdown table: the time, the bytes the counters saw per dispatch
(FETCH_SIZE doubled on gfx950 for wide reads, MI355X_MICROARCH.md §HBM) and the L2 hit rate.

    python tools/pmc_summary.py <dir with trace/ fetch/ write/ hit/ subdirectories>
"""
import collections
import csv
import glob
import os
import re
import sys


def short(name):
    name = name.replace("gnnrec::(anonymous namespace)::", "").replace("void ", "", 1)
    return re.sub(r"\(.*", "", name)


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def main(d):
    dur = collections.defaultdict(list)
    for r in rows(os.path.join(d, "trace", "**", "*kernel_stats.csv")):
        dur[short(r["Name"])] = (int(r["Calls"]), float(r["AverageNs"]) / 1e3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("fetch", "write", "hit"):
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | calls | avg us | FETCH_SIZE x2 MB | WRITE_SIZE MB | L2 hit |")
    print("|---|---|---|---|---|---|")
    for k in sorted(ctr, key=lambda k: -(dur.get(k, (0, 0))[0] * dur.get(k, (0, 0))[1])):
        c = ctr[k]
        calls, avg = dur.get(k, (0, 0.0))
        mean = lambda n: sum(c[n]) / len(c[n]) if c.get(n) else float("nan")  # noqa: E731
        fetch = 2 * mean("FETCH_SIZE") / 1e3  # KB -> MB, doubled
        write = mean("WRITE_SIZE") / 1e3
        hit, miss = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
        rate = hit / (hit + miss) if hit == hit and miss == miss and hit + miss > 0 else float("nan")
        print(f"| {k} | {calls} | {avg:.1f} | {fetch:.1f} | {write:.1f} | {rate:.3f} |")


if __name__ == "__main__":
    main(sys.argv[1])
