"""Median k_orth_chol duration split by its position within a step (P pass orth, Q pass orth),
over the last N orth launches of a rocprofv3 kernel trace. usage: kt_orth_pq.py <dir> [last]"""
import csv
import glob
import statistics
import sys

rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])))
rows = sorted((r for r in rows if 'k_orth_chol' in r['Kernel_Name']), key=lambda r: int(r['Start_Timestamp']))
rows = rows[-(int(sys.argv[2]) if len(sys.argv) > 2 else 40):]
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows]
n = {r['Kernel_Name'].split('(')[0].replace('void ', '') for r in rows}
print(f"first {statistics.median(d[0::2]):.2f}  second {statistics.median(d[1::2]):.2f}  {sorted(n)}")
