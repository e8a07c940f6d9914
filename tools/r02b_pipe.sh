#!/bin/bash
# even-product A/B: default vs software-pipelined build, over tile sizes (cold, kernel trace)
set -o pipefail
O=${1:-gpurun_out/pipe}; mkdir -p $O
export TMPDIR=/tmp
for v in "" pipe; do
  lib=$PWD/powersgd_amd/_lib${v:+_$v}/libpsgd.so
  for te in 8192 16384 32768; do
    for c in cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
      d=$O/${v:-default}_${te}_$c
      PSGD_LIB_PATH=$lib PSGD_TILE_ELEMS=$te timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- \
        python3 bench.py --config $c --steps 30 --warmup 4 --mode cold --no-cpu-baseline > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
      ms=$(python3 -c "import json;print(json.load(open('$d.json'))['ms_per_step'])")
      echo "${v:-default} $te $c ms=$ms $(python3 tools/prof_summary.py $d | grep -E 'k_product|k_reduce' | awk '{printf "%s %s | ", $1" "$2, $(NF-2)}')"
    done
  done
done
