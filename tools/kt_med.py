"""Median duration per kernel name over the last N launches of a rocprofv3 kernel trace.
usage: python tools/kt_med.py <dir> [last]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])))
rows = [r for r in rows if 'psgd' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 40
d = defaultdict(list)
for r in rows[-last:]:
    d[r['Kernel_Name'].split('(')[0].replace('void ', '')[:48]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
print("  ".join(f"{k} {statistics.median(v):.2f}" for k, v in d.items()))
