#!/bin/bash
# usage: tools/sweep.sh <config> "ENV=a ENV2=b" "ENV=c" ...   -> value ms_per_step final-pass-us per setting
cfg=$1; shift
for v in "$@"; do
  printf '%-40s ' "$v"
  env $v timeout -k 5 60 python bench.py --config "$cfg" --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" || exit 1
done
