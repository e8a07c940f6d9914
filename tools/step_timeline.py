"""Timeline of the last step(s) of a rocprofv3 --kernel-trace --hip-runtime-trace run: kernels (queue,
start, duration, gap to the previous kernel end on any queue) and the HIP API calls issued meanwhile.
usage: python tools/step_timeline.py <dir> [kernels_back] [api_filter,...]"""
import csv
import glob
import sys

d = sys.argv[1]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 12
kt = list(csv.DictReader(open(glob.glob(d + '/**/*kernel_trace.csv', recursive=True)[0])))
api = list(csv.DictReader(open(glob.glob(d + '/**/*hip_api_trace.csv', recursive=True)[0])))
kt.sort(key=lambda r: int(r['Start_Timestamp']))
ks = kt[-back:]
t0 = int(ks[0]['Start_Timestamp'])
t1 = int(ks[-1]['End_Timestamp'])
ev = []
prev_end = None
for r in ks:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    prev_end = e if prev_end is None else max(prev_end, e)
    ev.append((s, f"K q{r['Queue_Id']} {(s - t0) / 1e3:8.2f} +{(e - s) / 1e3:6.2f} gap {gap:6.2f}  {r['Kernel_Name'][:70]}"))
flt = sys.argv[3].split(',') if len(sys.argv) > 3 else None
for r in api:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    if s < t0 - 200000 or s > t1:
        continue
    if flt and not any(f in r['Function'] for f in flt):
        continue
    ev.append((s, f"A    {(s - t0) / 1e3:8.2f} +{(e - s) / 1e3:6.2f}            {r['Function']}"))
ev.sort()
for _, line in ev:
    print(line)
print(f"span {(t1 - t0) / 1e3:.2f} us over {len(ks)} kernels")
