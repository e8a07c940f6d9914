"""Per-kernel durations (last launches) from a rocprofv3 kernel trace, grouped by kernel name.
usage: python tools/kt_quick.py <dir> [substring]"""
import csv, glob, sys, statistics
from collections import defaultdict
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + '/**/*kernel_trace.csv', recursive=True)[0])))
filt = sys.argv[2] if len(sys.argv) > 2 else ""
rows.sort(key=lambda r: int(r['Start_Timestamp']))
seq = [(r['Kernel_Name'].split('(')[0][:60], (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3) for r in rows if filt in r['Kernel_Name']]
for i in range(0, len(seq), 20):
    chunk = seq[i:i + 20]
    print(f"{chunk[0][0]:60s}", " ".join(f"{d:.1f}" for _, d in chunk[-6:]))
