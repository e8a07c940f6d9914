"""Kernel sequence of the last steps of a rocprofv3 kernel trace: per dispatch its start
offset from the first shown dispatch, duration and the gap since the previous one (us).
usage: python tools/kt_seq.py <dir> [ndispatches] [all]"""
import csv
import glob
import sys

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
if not (len(sys.argv) > 3 and sys.argv[3] == "all"):  # "all": RCCL and torch kernels too
    rows = [r for r in rows if 'psgd' in r['Kernel_Name'] or 'rocclr' in r['Kernel_Name']]
rows = rows[-n:]
t0 = int(rows[0]['Start_Timestamp'])
prev = None
for r in rows:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} gap {gap:6.2f}  {r['Kernel_Name'].split('(')[0][:70]}")
    prev = e
