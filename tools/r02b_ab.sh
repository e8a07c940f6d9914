#!/bin/bash
# library-variant A/B (cold kernel traces + ms/step), variants given as _lib suffixes ("" = default)
set -o pipefail
O=${O:-gpurun_out/ab}; mkdir -p $O
export TMPDIR=/tmp
CFGS=${CFGS:-"cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16"}
for rep in 1 2; do
for v in "$@"; do
  lib=$PWD/powersgd_amd/_lib${v:+_$v}/libpsgd.so
  for c in $CFGS; do
    d=$O/${v:-default}_${c}_$rep
    PSGD_LIB_PATH=$lib timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- \
      python3 bench.py --config $c --steps 30 --warmup 4 --mode cold --no-cpu-baseline > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
    ms=$(python3 -c "import json;print(json.load(open('$d.json'))['ms_per_step'])")
    echo "${v:-default} $c ms=$ms $(python3 tools/prof_summary.py $d | grep -E 'psgd' | awk '{printf "%s %s | ", $1" "$2, $(NF-2)}')"
  done
done
done
