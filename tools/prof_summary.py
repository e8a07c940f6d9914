"""Summarise rocprofv3 CSV output: per-kernel average duration, launch count, idle gaps,
and per-kernel PMC averages (FETCH_SIZE / WRITE_SIZE, KB per dispatch).

usage: python tools/prof_summary.py <rocprofv3 output dir> [--traffic CFG]

--traffic CFG: also merge the per-launch HBM traffic of the final pass (k_final_odd, else
k_apply; FETCH_SIZE x 2, the gfx950
16-B streaming-read correction of MI355X_MICROARCH.md §HBM, + WRITE_SIZE; KB -> bytes) into
profiles/pmc_traffic.json under key CFG (read by bench.py for roofline.traffic).
"""
import json
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
    traffic = {}
    for path in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        rows = list(csv.DictReader(open(path)))
        acc = defaultdict(list)
        for r in rows:
            acc[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        print(f"# {path}")
        for (k, c), v in sorted(acc.items()):
            print(f"{k[:70]:70s} {c:12s} n={len(v):4d} avg={statistics.mean(v):14.1f}")
            # the final pass: k_final_odd / k_final_proj (fused last odd iteration) if the run has it, else k_apply
            if k.startswith(("psgd::k_final_odd", "psgd::k_final_proj", "psgd::k_apply")) and c in ("FETCH_SIZE", "WRITE_SIZE"):
                prio = 2 if k.startswith(("psgd::k_final_odd", "psgd::k_final_proj")) else 1
                if prio >= traffic.get(c + "_prio", 0):
                    traffic[c] = statistics.mean(v) * 1024 * (2 if c == "FETCH_SIZE" else 1)
                    traffic[c + "_prio"] = prio
    if "--traffic" in sys.argv and "FETCH_SIZE" in traffic and "WRITE_SIZE" in traffic:
        cfg = sys.argv[sys.argv.index("--traffic") + 1]
        # on the GPU box only gpurun_out/ travels back: write there (tools/merge_traffic.py
        # folds it into the committed profiles/pmc_traffic.json)
        out = os.environ.get("PSGD_TRAFFIC_OUT") or os.path.join(
            os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "pmc_traffic.json")
        try:
            data = json.load(open(out))
        except (OSError, ValueError):
            data = {}
        data[cfg] = round(traffic["FETCH_SIZE"] + traffic["WRITE_SIZE"])
        json.dump(data, open(out, "w"), indent=1, sort_keys=True)
        print(f"k_apply HBM traffic per launch: {data[cfg]} B (FETCH x2 + WRITE) -> {out}")


if __name__ == "__main__":
    main()
