#!/bin/bash
out=$1; mkdir -p $out; export TMPDIR=/tmp
for w in single resnet50; do for r in 1 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $out/kt_${w}_$r -o kt -- python3 tools/even_alone.py $w $r 30 > $out/${w}_$r.log 2>&1 || exit 1
  python3 - $out/kt_${w}_$r $w $r <<'PY'
import csv, glob, statistics, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))
for name in ("k_even", "k_reduce"):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
    print(sys.argv[2], sys.argv[3], name, f"median {statistics.median(d[-20:]):.2f} us min {min(d[-20:]):.2f}")
PY
done; done
