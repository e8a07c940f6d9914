#!/bin/bash
# small plans: final-pass block size and product tile size sweeps (cold ms/step, no profiler)
set -o pipefail
O=gpurun_out/small; mkdir -p $O
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4; do
  for fe in 0 1024 2048 8192; do
    for te in 0 1024 2048 8192; do
      env_fe=""; [ $fe != 0 ] && env_fe="PSGD_FIN_ELEMS=$fe"
      env_te=""; [ $te != 0 ] && env_te="PSGD_TILE_ELEMS=$te"
      env $env_fe $env_te timeout -k 10 60 python3 bench.py --config $c --steps 200 --warmup 20 --mode cold --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
      echo "$c fin_elems=$fe tile_elems=$te $(python3 -c "import json;d=json.load(open('$O/b.json'));print(d['ms_per_step'], d['roofline']['avg_launch_us'])")"
    done
  done
done
