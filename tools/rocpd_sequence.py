"""The kernels of the last `n` launches before the closing torch.cuda._sleep marker of a
rocprofv3 rocpd trace, in launch order with durations (one replay of a captured step:
which launch of which op costs what).

    python tools/rocpd_sequence.py <run>_results.db n
"""
import re
import sqlite3
import sys


def main(path: str, n: int) -> None:
    db = sqlite3.connect(path)
    rows = db.execute("select start, end, name from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if "spin_kernel" in r[2]]
    end = marks[-1] if marks else len(rows)
    seq = rows[max(0, end - n):end]
    t0 = seq[0][0]
    tot = 0
    for s, e, name in seq:
        name = re.sub(r"\(.*", "", name.replace("gnnrec::(anonymous namespace)::", "")
                      .replace("void ", "", 1))[:100]
        tot += e - s
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.2f}  {name}")
    print(f"sum {tot / 1e3:.1f} us over {len(seq)} kernels, span {(seq[-1][1] - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
