"""Plain-step kernel trace summary (tools/step_trace.py under rocprofv3 --kernel-trace): per psgd
kernel its median duration over the last `last` dispatches, the median gap between consecutive
psgd dispatches, and the median step period (start to start of the step's first kernel name).
usage: python tools/kt_steps.py <dir> [last]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])))
rows = [r for r in rows if 'psgd' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 120
rows = rows[-last:]
name = lambda r: r['Kernel_Name'].split('(')[0].replace('void ', '')[:48]
d = defaultdict(list)
for r in rows:
    d[name(r)].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
gaps = [(int(b['Start_Timestamp']) - int(a['End_Timestamp'])) / 1e3 for a, b in zip(rows, rows[1:])]
first = name(rows[0])
starts = [int(r['Start_Timestamp']) for r in rows if name(r) == first]
period = statistics.median([(b - a) / 1e3 for a, b in zip(starts, starts[1:])]) if len(starts) > 1 else 0.0
print("  ".join(f"{k} {statistics.median(v):.2f}" for k, v in d.items()) +
      f"  | gap_med {statistics.median(gaps):.2f} gap_sum/step {sum(gaps) / max(len(starts), 1):.2f} period {period:.2f}")
