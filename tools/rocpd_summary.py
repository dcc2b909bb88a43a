"""Per-kernel statistics out of a rocprofv3 database (the default `--kernel-trace --stats`
output, <name>_results.db): calls, total / average µs and share, as a markdown table.

    python tools/rocpd_summary.py <results.db> [top=30] > profiles/<tag>_kernel_stats.md
"""
import re
import sqlite3
import sys


def short(name: str) -> str:
    """Kernel name without argument lists and namespaces (template arguments kept)."""
    n = re.sub(r"\(.*$", "", name.replace("(anonymous namespace)::", ""))
    n = n.replace("gnnrec::", "").replace("void ", "")
    return n if len(n) < 110 else n[:107] + "..."


def main():
    db, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 30
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage "
                          "from top_kernels"))
    tot = sum(r[2] for r in rows)
    print(f"rocprofv3 --kernel-trace --stats: {len(rows)} kernels, {sum(r[1] for r in rows)} "
          f"dispatches, {tot / 1e3:.3f} ms of kernel time\n")
    print("| kernel | calls | total µs | avg µs | share |")
    print("|---|---|---|---|---|")
    for name, calls, total, avg, pct in rows[:top]:
        print(f"| `{short(name)}` | {calls} | {total:.1f} | {avg:.3f} | {pct:.1f} % |")


if __name__ == "__main__":
    main()
