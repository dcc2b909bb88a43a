"""Kernel statistics (calls, total / average duration in us, share) from a rocprofv3 rocpd
database (the tool's default output format) as CSV, names shortened to the kernel symbol —
the same columns as `rocprofv3 --stats`' kernel_stats.csv.

    python tools/rocpd_stats.py gpurun_out/<run>/<dir>/<name>_results.db > profiles/<x>.csv
"""
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("gnnrec::(anonymous namespace)::", "").replace("void ", "", 1)
    return name[:160] if name.startswith("at::") else re.sub(r"\(.*", "", name)


def main(path: str, limit: int = 60) -> None:
    db = sqlite3.connect(path)
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "Percentage"])
    for name, calls, tot, avg, pct in db.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"
            f" limit {int(limit)}"):
        w.writerow([short(name), calls, f"{tot:.3f}", f"{avg:.3f}", f"{pct:.2f}"])


if __name__ == "__main__":
    main(*sys.argv[1:2])
