"""Durations of one kernel, in dispatch order, from a rocprofv3 kernel trace (which launch of a
rotating-set / alternating-parity loop is slow?). usage: python tools/kt_series.py <dir> <substring>"""
import csv
import glob
import sys

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])))
rows = [r for r in rows if sys.argv[2] in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
print(f"{sys.argv[2]}: {len(d)} launches")
for i in range(0, len(d), 8):
    print(f"{i:4d}: " + " ".join(f"{x:6.2f}" for x in d[i:i + 8]))
