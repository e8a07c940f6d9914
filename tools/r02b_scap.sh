#!/bin/bash
set -o pipefail
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg2_resnet50_r1; do
  for sc in 0 2 3 5; do
    env_sc=""; [ $sc != 0 ] && env_sc="PSGD_FIN_SCAP=$sc"
    env $env_sc timeout -k 10 60 python3 bench.py --config $c --steps 200 --warmup 20 --mode cold --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    echo "$c scap=$sc $(python3 -c "import json;d=json.load(open('gpurun_out/b.json'));print(d['ms_per_step'], d['roofline']['avg_launch_us'])")"
  done
done
PSGD_FIN_SCAP=5 timeout -k 10 300 python -u -m pytest tests/test_gpu_final.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1
