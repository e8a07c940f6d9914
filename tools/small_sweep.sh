#!/bin/bash
# cfg5 (small plan) block-size sweep: K-term / odd-even row blocks (PSGD_FIN_ELEMS_KT) and even-product
# range size (PSGD_EVEN_MIN) around the defaults (8192 / 16384), bench ms per step, two passes. GPU box.
mkdir -p gpurun_out/r06r
for rep in 1 2; do
for fe in 8192 2048 4096 16384; do
  PSGD_FIN_ELEMS_KT=$fe timeout -k 10 100 python bench.py --config cfg5_lstm_r1_i4 --steps 200 --warmup 20 --mode cold --no-cpu-baseline --no-extra > gpurun_out/r06r/fe$fe.json 2>/dev/null || exit 1
  echo "rep$rep fin_elems_kt=$fe $(python3 -c "import json;d=json.load(open('gpurun_out/r06r/fe$fe.json'));print(d['ms_per_step'])")"
done
for em in 4096 8192 32768; do
  PSGD_EVEN_MIN=$em timeout -k 10 100 python bench.py --config cfg5_lstm_r1_i4 --steps 200 --warmup 20 --mode cold --no-cpu-baseline --no-extra > gpurun_out/r06r/em$em.json 2>/dev/null || exit 1
  echo "rep$rep even_min=$em $(python3 -c "import json;d=json.load(open('gpurun_out/r06r/em$em.json'));print(d['ms_per_step'])")"
done
done
