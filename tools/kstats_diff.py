"""Per-iteration kernel budget from two rocprofv3 kernel_stats.csv files of the same
program run for N1 and N2 iterations: (totals2 - totals1) / (N2 - N1) per kernel.

    python tools/kstats_diff.py stats_N1.csv stats_N2.csv N2-N1
"""
import csv
import sys


def load(path):
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"]))
            for r in csv.DictReader(open(path))}


def main():
    a, b, n = load(sys.argv[1]), load(sys.argv[2]), int(sys.argv[3])
    rows = []
    for name, (c2, t2) in b.items():
        c1, t1 = a.get(name, (0, 0.0))
        if c2 - c1 > 0:
            rows.append(((t2 - t1) / n / 1e3, (c2 - c1) / n, name))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"per iteration: {tot:.1f} us over {sum(r[1] for r in rows):.1f} launches")
    for us, calls, name in rows:
        print(f"{us:8.2f} us {calls:6.2f} x  {us / calls:7.2f} us  {name[:120]}")


if __name__ == "__main__":
    main()
