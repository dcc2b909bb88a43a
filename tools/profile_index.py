"""Regenerate the per-prefix file list of profiles/INDEX.md ("## Current files" bullets)
from the files present; the text above the bullets and the "## Removed" section stay.

    python tools/profile_index.py
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def main():
    path = os.path.join(PROF, "INDEX.md")
    text = open(path).read()
    head, rest = text.split("\n* **", 1)
    removed = rest[rest.index("\n## Removed"):]
    groups = {}
    for f in sorted(os.listdir(PROF)):
        if f == "INDEX.md" or f.startswith("."):
            continue
        m = re.match(r"(p1|r\d\d[a-z0-9]*)_", f)
        groups.setdefault(m.group(1) if m else "other", []).append(f)

    def key(k):
        m = re.match(r"r(\d\d)([a-z0-9]*)", k)
        if k == "p1" or m is None:
            return (0 if k == "p1" else 2, 0, 0, k)
        return (1, int(m.group(1)), len(m.group(2)), m.group(2))
    lines = [f"* **{k}**: " + ", ".join(f"`{f}`" for f in groups[k])
             for k in sorted(groups, key=key)]
    open(path, "w").write(head.rstrip("\n") + "\n\n" + "\n".join(lines) + "\n" + removed)


if __name__ == "__main__":
    main()
