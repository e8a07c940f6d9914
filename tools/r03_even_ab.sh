#!/bin/bash
# A/B of the persistent even product (k_even): library variant x workgroups per CU, cold
# ResNet-50 rank 1 / rank 4; per run the k_even / k_reduce kernel times (rocprofv3 kernel trace)
# and the un-profiled step time. usage: tools/r03_even_ab.sh <out> "<lib>:<ENV=v,ENV=v> ..."
out=$1; shift
export TMPDIR=/tmp
mkdir -p "$out"
for spec in $@; do
  lib=${spec%%:*}; envs=${spec##*:}
  for cfg in ${AB_CONFIGS:-cfg2_resnet50_r1 cfg3_resnet50_r4}; do
    tag=$(basename $(dirname $lib))_$(echo $envs | tr ',=' '__')_$cfg
    (
      export PSGD_LIB_PATH=$PWD/$lib
      for e in ${envs//,/ }; do export $e; done
      timeout -k 10 120 python3 bench.py --config $cfg --steps 40 --warmup 10 --mode cold --no-cpu-baseline --no-extra > "$out/$tag.json" 2> "$out/$tag.err" || exit 1
      timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "/tmp/kt_$tag" -o kt -- python3 bench.py --config $cfg --steps 20 --warmup 4 --mode cold --no-cpu-baseline --no-extra > /dev/null 2>&1 || exit 1
    ) || exit 1
    python3 - "$out" "$tag" <<'PY'
import csv, glob, json, statistics, sys
out, tag = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(f"/tmp/kt_{tag}/**/*kernel_trace.csv", recursive=True)[0])))
def avg(name):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if name in r["Kernel_Name"]]
    return statistics.median(d[-16:]) if d else float("nan")
ms = json.load(open(f"{out}/{tag}.json"))["ms_per_step"]
print(f"{tag:60s} step {ms*1e3:7.1f} us  k_even {avg('k_even'):6.2f}  k_reduce {avg('k_reduce'):5.2f}  final {avg('k_final'):6.2f}")
PY
  done
done
