#!/bin/bash
# k_even alone (tools/even_alone.py) under library variants: kernel-trace medians of k_even.
export TMPDIR=/tmp
for lib in "$@"; do
  for spec in "single 1" "single 4" "resnet50 1" "resnet50 4"; do
    tag=$(basename $(dirname $lib))_${spec// /_}
    PSGD_LIB_PATH=$PWD/$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/ed_$tag -o kt -- python3 tools/even_alone.py $spec 24 > /dev/null 2>&1 || { echo "$tag failed"; exit 1; }
    python3 - "$tag" <<'PY'
import csv, glob, statistics, sys
tag = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(f"/tmp/ed_{tag}/**/*kernel_trace.csv", recursive=True)[0])))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if "k_even" in r["Kernel_Name"]]
print(f"{tag:40s} k_even median {statistics.median(d[-16:]):7.2f} us  min {min(d[-16:]):7.2f}")
PY
  done
done
