"""GPU busy fraction of the C2 probe's timed steps from a rocprofv3 kernel trace.

    python tools/c2_busy.py <kernel_trace.csv> <wall_ms_per_step> [steps=20]

The timed window is the trace's last steps x wall_ms (the probe times its last 20 steps and
launches nothing after them); busy = the union of kernel intervals inside it.  Prints the
per-step kernel time, the busy fraction and the top kernels of the window."""
import csv
import sys
from collections import defaultdict


def main():
    path, wall = sys.argv[1], float(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
            for r in csv.DictReader(open(path))]
    rows.sort()
    end = max(e for _, e, _ in rows)
    lo = end - steps * wall * 1e6
    win = [(max(s, lo), e, n) for s, e, n in rows if e > lo]
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    per = defaultdict(lambda: [0, 0])
    for s, e, n in win:
        per[n][0] += 1
        per[n][1] += e - s
    tot = sum(v[1] for v in per.values())
    print(f"window {steps} steps x {wall:.3f} ms: kernels {len(win) / steps:.0f}/step, "
          f"kernel time {tot / 1e6 / steps:.3f} ms/step, busy {busy / 1e6 / steps:.3f} ms/step "
          f"= {busy / (steps * wall * 1e6):.2f} of wall")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"{c / steps:6.1f}/step {t / 1e3 / steps:8.1f} us/step  {n[:110]}")


if __name__ == "__main__":
    main()
