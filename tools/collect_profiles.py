"""Copy one profile_round.sh run out of gpurun_out/ into profiles/ (the committed record):

    python tools/collect_profiles.py <tag>

gpurun_out/<tag>_trace/**/*kernel_stats.csv -> profiles/<tag>_kernel_stats.csv, the PMC
passes' *counter_collection.csv -> profiles/<tag>_pmc_{fetch,write,dram,mfma}.csv, the
meta json, the trace run's bench line, the last pass's kernel timeline (tools/timeline.py)
and the roofline digest (tools/summarize_profiles.py)."""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
OUT, PROF = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")


def one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"nothing matches {pattern}")
    return hits[-1]


def main(tag):
    shutil.copy(one(f"{OUT}/{tag}_trace/**/*kernel_stats.csv"), f"{PROF}/{tag}_kernel_stats.csv")
    for kind in ("fetch", "write", "dram", "mfma"):
        src = glob.glob(f"{OUT}/{tag}_{kind}/**/*counter_collection.csv", recursive=True)
        if src:
            shutil.copy(sorted(src)[-1], f"{PROF}/{tag}_pmc_{kind}.csv")
    shutil.copy(f"{OUT}/{tag}_pmc_meta.json", f"{PROF}/{tag}_pmc_meta.json")
    line = [ln for ln in open(f"{OUT}/{tag}_trace.log") if ln.startswith("{")]
    if line:
        open(f"{PROF}/{tag}_trace_bench_line.json", "w").write(line[-1])
    trace = one(f"{OUT}/{tag}_trace/**/*kernel_trace.csv")
    tl = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "timeline.py"), trace],
                        capture_output=True, text=True, check=True).stdout
    open(f"{PROF}/{tag}_timeline.txt", "w").write(tl)
    sm = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "summarize_profiles.py"),
                         tag], capture_output=True, text=True, check=True).stdout
    open(f"{PROF}/{tag}_summary.md", "w").write(sm)
    print(f"profiles/{tag}_*: stats, {len(glob.glob(f'{PROF}/{tag}_pmc_*.csv'))} PMC files, "
          f"timeline, summary")


if __name__ == "__main__":
    main(sys.argv[1])
