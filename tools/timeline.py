"""Kernel timeline of one full-graph pass from a rocprofv3 kernel trace.

    python tools/timeline.py gpurun_out/<dir>/<...>_kernel_trace.csv [--last-ms 400]

Prints the kernels of the last pass (names shortened) with start/end offsets, and the
time the GPU had no kernel running (gaps) vs. the time two kernels overlapped.
"""
import csv
import sys


def short(name):
    n = name.split("(anonymous namespace)::", 1)[-1]
    return n.split("(")[0][:60]


def main(path, window_ms=None):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in rows)
    gnn = [e for e in ev if "gnnrec" in e[2] or "spmm" in e[2] or "gemm" in e[2]]
    # the last pass: from the last synth-free run of spmm/gemm launches; take a time window
    end = max(e[1] for e in gnn)
    if window_ms is None:
        window_ms = 400.0
    t0 = end - int(window_ms * 1e6)
    sel = [e for e in ev if e[0] >= t0]
    base = sel[0][0]
    busy, last_end, overlap = 0, base, 0
    for s, e, n in sel:
        print(f"{(s - base) / 1e6:9.3f} {(e - base) / 1e6:9.3f} {(e - s) / 1e6:8.3f}  {n}")
        if s > last_end:
            busy += e - s
        else:
            overlap += min(e, last_end) - s
            busy += max(0, e - last_end)
        last_end = max(last_end, e)
    span = last_end - base
    print(f"span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(span - busy) / 1e6:.3f} ms,"
          f" overlapped {overlap / 1e6:.3f} ms")


if __name__ == "__main__":
    w = None
    if "--last-ms" in sys.argv:
        w = float(sys.argv[sys.argv.index("--last-ms") + 1])
    main(sys.argv[1], w)
