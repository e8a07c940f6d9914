#!/bin/bash
set -o pipefail
O=gpurun_out/small2; mkdir -p $O
for c in cfg5_lstm_r1_i4 cfg1_1024sq_r1; do
  for fe in 4096 8192 16384 32768; do
    for te in 8192 16384 32768 65536; do
      PSGD_FIN_ELEMS=$fe PSGD_TILE_ELEMS=$te timeout -k 10 60 python3 bench.py --config $c --steps 200 --warmup 20 --mode cold --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
      echo "$c fin_elems=$fe tile_elems=$te $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['ms_per_step'], d['roofline']['avg_launch_us'])")"
    done
  done
done
