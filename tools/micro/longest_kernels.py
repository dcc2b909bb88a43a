"""Longest kernels of a rocprofv3 kernel trace: python longest_kernels.py <trace.csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 8
ev = sorted(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
             r["Kernel_Name"].split("(anonymous namespace)::")[-1][:70], r.get("Stream_Id", ""))
            for r in rows)
for d, k, s in ev[-n:]:
    print(f"{d:10.3f} ms  stream {s}  {k}")
