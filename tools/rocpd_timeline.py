"""GPU occupancy of a kernel trace's steady state, from a rocprofv3 rocpd database: between
the first and last torch.cuda._sleep marker kernel (spin_kernel), else over the middle `frac`
of the traced span, the union of
kernel intervals (busy time), the summed kernel time (> busy where kernels overlap), the
idle gaps by size, and the busiest queues — whether a loop is GPU-bound, host-bound or
serialised across streams.

    python tools/rocpd_timeline.py <run>_results.db [frac=0.6]
"""
import json
import sqlite3
import sys


def main(path: str, frac: float = 0.6) -> None:
    db = sqlite3.connect(path)
    cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
    q = "queue_id" if "queue_id" in cols else ("stream_id" if "stream_id" in cols else None)
    sel = f"select start, end, name{', ' + q if q else ''} from kernels order by start"
    rows = db.execute(sel).fetchall()
    if not rows:
        print(json.dumps({"error": "no kernels", "columns": cols}))
        return
    marks = [r for r in rows if "spin_kernel" in r[2]]
    if len(marks) >= 2:  # the probe's torch.cuda._sleep markers bracket the timed loop
        w0, w1 = marks[0][1], marks[-1][0]
        rows = [r for r in rows if "spin_kernel" not in r[2]]
    else:
        t_first, t_last = rows[0][0], max(r[1] for r in rows)
        span = t_last - t_first
        w0 = t_first + span * (1 - frac) / 2
        w1 = w0 + span * frac
    win = [r for r in rows if r[0] >= w0 and r[1] <= w1]
    busy, summed, gaps, cur_end = 0, 0, [], None
    per_q = {}
    for r in win:
        s, e = r[0], r[1]
        summed += e - s
        if q:
            per_q[r[3]] = per_q.get(r[3], 0) + (e - s)
        if cur_end is None or s > cur_end:
            if cur_end is not None:
                gaps.append(s - cur_end)
            busy += e - s
            cur_end = e
        elif e > cur_end:
            busy += e - cur_end
            cur_end = e
    wall = w1 - w0
    edges = [2e3, 5e3, 20e3, 100e3]
    hist = {f"<{int(b / 1e3)}us": 0 for b in edges}
    hist[">=100us"] = 0
    gap_time = {k: 0 for k in hist}
    for g in gaps:
        for b in edges:
            if g < b:
                hist[f"<{int(b / 1e3)}us"] += 1
                gap_time[f"<{int(b / 1e3)}us"] += g
                break
        else:
            hist[">=100us"] += 1
            gap_time[">=100us"] += g
    print(json.dumps({
        "window_ms": round(wall / 1e6, 3), "kernels": len(win),
        "busy_frac": round(busy / wall, 4), "summed_over_wall": round(summed / wall, 4),
        "idle_gaps": hist, "idle_ms_by_gap": {k: round(v / 1e6, 3) for k, v in gap_time.items()},
        "queues": {str(k): round(v / 1e6, 3) for k, v in
                   sorted(per_q.items(), key=lambda kv: -kv[1])[:6]},
    }))


if __name__ == "__main__":
    main(sys.argv[1], *(float(a) for a in sys.argv[2:3]))
