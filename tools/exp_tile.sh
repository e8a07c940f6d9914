#!/bin/bash
# even product / full step vs PSGD_TILE_ELEMS (cold)
export TMPDIR=/tmp
O=gpurun_out/tile; mkdir -p $O
for te in 4096 8192 12288 16384 32768; do
  for spec in "cfg3_resnet50_r4" "cfg2_resnet50_r1"; do
    d=$O/${te}_${spec}
    PSGD_TILE_ELEMS=$te timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o kt -- python3 tools/exp_even.py $spec even > $d.log 2>&1 || exit 1
    echo "== $te $spec $(python3 tools/prof_summary.py $d | grep -E 'k_product|k_reduce' | awk '{printf "%s %s  ", $1, $(NF-2)}')"
  done
  PSGD_TILE_ELEMS=$te timeout -k 10 100 python3 bench.py --config cfg3_resnet50_r4 --no-cpu-baseline --steps 50 > $O/b3_$te.json || exit 1
  PSGD_TILE_ELEMS=$te timeout -k 10 100 python3 bench.py --config cfg2_resnet50_r1 --no-cpu-baseline --steps 50 > $O/b2_$te.json || exit 1
  python3 -c "import json; a=json.load(open('$O/b3_$te.json')); b=json.load(open('$O/b2_$te.json')); print('bench $te cfg3', a['ms_per_step'], a['warm']['ms_per_step'], 'cfg2', b['ms_per_step'], b['warm']['ms_per_step'])"
done
