"""Summarise rocprofv3 CSV output: per-kernel average duration, launch count, idle gaps,
and per-kernel PMC averages (FETCH_SIZE / WRITE_SIZE, KB per dispatch).

usage: python tools/prof_summary.py <rocprofv3 output dir> [kernel-substring-filter]
"""
import csv
import glob
import os
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").strip()


def main():
    d = sys.argv[1]
    kt = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))
    for path in kt:
        rows = list(csv.DictReader(open(path)))
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        by = defaultdict(list)
        for r in rows:
            by[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print(f"# {path}: {len(rows)} dispatches")
        print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>9s} {'med_us':>9s} {'total_us':>10s}")
        for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            print(f"{k[:70]:70s} {len(v):6d} {statistics.mean(v):9.2f} {statistics.median(v):9.2f} {sum(v):10.1f}")
        gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rows, rows[1:])]
        small = [g for g in gaps if 0 <= g < 50]
        if small:
            print(f"gaps<50us between consecutive dispatches: n={len(small)} mean={statistics.mean(small):.2f} us "
                  f"median={statistics.median(small):.2f} us")
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        rows = list(csv.DictReader(open(path)))
        acc = defaultdict(list)
        for r in rows:
            acc[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        print(f"# {path}")
        for (k, c), v in sorted(acc.items()):
            print(f"{k[:70]:70s} {c:12s} n={len(v):4d} avg={statistics.mean(v):14.1f}")


if __name__ == "__main__":
    main()
