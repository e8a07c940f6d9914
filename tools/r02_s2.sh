#!/bin/bash
# round-2 session 2: host overhead after the native output slab; cold-cache tile sweep
tools/gpu_steps.sh \
  "t_slab|300|python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread" \
  "bench_cfg2|200|python bench.py --no-cpu-baseline" \
  "bench_cfg3|200|python bench.py --config cfg3_resnet50_r4 --no-cpu-baseline" \
  "bench_cfg1|200|python bench.py --config cfg1_1024sq_r1 --no-cpu-baseline" \
  "bench_cfg5|200|python bench.py --config cfg5_lstm_r1_i4 --no-cpu-baseline" \
  "bench_cfg4|200|python bench.py --config cfg4_llama_r2_bf16 --no-cpu-baseline" \
  "sweep|400|for t in 8192 32768 65536; do echo tile=\$t; PSGD_TILE_ELEMS=\$t timeout -k 5 60 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sw\$t -o kt -- python3 bench.py --steps 40 --warmup 4 --mode cold --no-cpu-baseline > /dev/null 2>&1 || exit 1; python3 tools/prof_summary.py gpurun_out/sw\$t | head -6; done"
exit 0
