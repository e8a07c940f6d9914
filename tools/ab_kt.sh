#!/bin/bash
# A/B kernel medians: for each library variant (default build = "base", or _lib_v/<name>) and
# config, a rocprofv3 kernel trace of plain cold steps (tools/step_trace.py -> tools/kt_steps.py)
# and the un-profiled bench line of the same config. Variants run
# interleaved (base, v1, ..., base, v1, ...) `reps` times so box drift hits every side.
# usage: tools/ab_kt.sh <outdir> <reps> "<cfgs>" <variant>...   (GPU box)
out=$1; reps=$2; cfgs=$3; shift 3
mkdir -p "$out"
export TMPDIR=/tmp
for rep in $(seq 1 "$reps"); do
  for v in "$@"; do
    if [ "$v" = base ]; then lib=""; else lib="$PWD/powersgd_amd/_lib_v/$v/libpsgd.so"; fi
    for cfg in $cfgs; do
      d="$out/$v.$cfg.$rep"
      PSGD_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$d" -o kt -- \
        python3 tools/step_trace.py "$cfg" 60 > "$d.log" 2>&1 || { echo "FAILED $v $cfg"; exit 1; }
      PSGD_LIB_PATH=$lib timeout -k 10 120 python3 bench.py --config "$cfg" --steps 100 --warmup 10 --mode cold \
        --no-cpu-baseline --no-extra > "$d.json" 2> "$d.err" || { echo "FAILED bench $v $cfg"; exit 1; }
      echo "$v $cfg rep$rep: $(python3 tools/kt_steps.py "$d" 150)  bench_ms=$(python3 -c "import json;print(json.load(open('$d.json'))['ms_per_step'])")" | tee -a "$out/summary.txt"
      rm -rf "$d"
    done
  done
done
