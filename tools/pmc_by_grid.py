"""Per (kernel, grid size) averages of a rocprofv3 kernel trace and its PMC passes — like
tools/pmc_summary.py, but dispatches of one kernel with different grids (the sampler's
pick / finalize of step 0 and step 1, sized by each step's capacities) are kept apart.

    python tools/pmc_by_grid.py <dir with trace/ fetch/ write/ hit/ subdirectories> [regex]

FETCH_SIZE is doubled on gfx950 for wide reads (MI355X_MICROARCH.md §HBM), as pmc_summary."""
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


def grid(r):
    for k in ("Grid_Size", "Grid_Size_X", "Grid_X"):
        if k in r and r[k] not in (None, ""):
            return int(r[k])
    return 0


def main(d, pat=None):
    rx = re.compile(pat) if pat else None
    dur = collections.defaultdict(list)
    for r in rows(os.path.join(d, "trace", "**", "*kernel_trace.csv")):
        k = short(r["Kernel_Name"])
        if rx and not rx.search(k):
            continue
        dur[(k, grid(r))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for sub in ("fetch", "write", "hit"):
        for r in rows(os.path.join(d, sub, "**", "*counter_collection.csv")):
            k = short(r["Kernel_Name"])
            if rx and not rx.search(k):
                continue
            ctr[(k, grid(r))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("| kernel | grid | calls | avg us | FETCH_SIZE x2 MB | WRITE_SIZE MB | L2 hit | TB/s |")
    print("|---|---|---|---|---|---|---|---|")
    keys = set(dur) | set(ctr)
    for key in sorted(keys, key=lambda k: -sum(dur.get(k, [0]))):
        ts = dur.get(key, [])
        avg = sum(ts) / len(ts) if ts else float("nan")
        c = ctr.get(key, {})
        mean = lambda n: sum(c[n]) / len(c[n]) if c.get(n) else float("nan")  # noqa: E731
        fetch = 2 * mean("FETCH_SIZE") / 1e3  # KB -> MB, doubled
        write = mean("WRITE_SIZE") / 1e3
        hit, miss = mean("TCC_HIT_sum"), mean("TCC_MISS_sum")
        rate = hit / (hit + miss) if hit == hit and miss == miss and hit + miss > 0 else float("nan")
        tbs = (fetch + write) / avg if avg == avg and avg > 0 else float("nan")  # MB/us
        print(f"| {key[0]} | {key[1]} | {len(ts)} | {avg:.1f} | {fetch:.1f} | {write:.1f} | "
              f"{rate:.3f} | {tbs:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
