#!/bin/bash
# A/B of library build variants: cold kernel trace of a bench config per variant.
# usage: tools/ab_libs.sh <config> <variant>...   (variant "" = default build)
cfg=$1; shift
export TMPDIR=/tmp
for v in "$@"; do
  lib=powersgd_amd/_lib${v:+_$v}/libpsgd.so
  out=gpurun_out/ab_${cfg}_${v:-default}
  PSGD_LIB_PATH=$PWD/$lib timeout -k 5 90 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o kt -- python3 bench.py --config $cfg --steps 40 --warmup 4 --mode cold --no-cpu-baseline > $out.log 2>&1 || exit 1
  echo "== $cfg ${v:-default}: $(grep -o '"ms_per_step": [0-9.]*' $out.log)"
  python3 tools/prof_summary.py $out > $out.txt; grep psgd $out.txt
done
