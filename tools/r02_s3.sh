#!/bin/bash
# round-2 session 3: full GPU suite (+ parity log), smoke, benches (all configs), cold rocprof of
# the headline config (kernel trace + FETCH/WRITE PMC) and cfg3
export PSGD_PARITY_LOG=gpurun_out/parity_errors.jsonl
rm -f $PSGD_PARITY_LOG gpurun_out/pmc_traffic.json
tools/gpu_steps.sh \
  "pytest|500|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_cfg2|240|python bench.py" \
  "bench_cfg3|200|python bench.py --config cfg3_resnet50_r4 --no-cpu-baseline" \
  "bench_cfg1|200|python bench.py --config cfg1_1024sq_r1 --no-cpu-baseline" \
  "bench_cfg5|200|python bench.py --config cfg5_lstm_r1_i4 --no-cpu-baseline" \
  "bench_cfg4|200|python bench.py --config cfg4_llama_r2_bf16 --no-cpu-baseline" \
  "prof_cfg2|400|tools/profile.sh cfg2_resnet50_r1 gpurun_out/prof_cfg2 cold" \
  "prof_cfg3|400|tools/profile.sh cfg3_resnet50_r4 gpurun_out/prof_cfg3 cold"
python3 tools/parity_summary.py $PSGD_PARITY_LOG > gpurun_out/parity_summary.json 2>/dev/null
exit 0
