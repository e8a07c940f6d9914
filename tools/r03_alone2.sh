#!/bin/bash
out=$1; mkdir -p $out; export TMPDIR=/tmp
for spec in "single 4 11 read" "single 4 4 read" "single 4 4 write" "single 4 4 step" "resnet50 4 4 step" "resnet50 1 4 step"; do
  set -- $spec; tag=$1_$2_$3_$4
  timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $out/kt_$tag -o kt -- python3 tools/even_alone.py $1 $2 30 $3 $4 > $out/$tag.log 2>&1 || exit 1
  python3 - $out/kt_$tag $tag <<'PY'
import csv, glob, statistics, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0])))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_even" in r["Kernel_Name"]]
print(f"{sys.argv[2]:28s} k_even median {statistics.median(d[-20:]):.2f} us min {min(d[-20:]):.2f}")
PY
done
