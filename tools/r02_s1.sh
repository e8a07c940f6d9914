#!/bin/bash
# round-2 GPU session 1: GPU tests (+ parity error log), smoke, bench cfg2/cfg3, stream-copy
# ceilings (warm + cold), rocprof kernel trace + PMC traffic of the cold cfg2 bench.
export PSGD_PARITY_LOG=gpurun_out/parity_errors.jsonl
rm -f $PSGD_PARITY_LOG
tools/gpu_steps.sh \
  "pytest|500|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_cfg2|240|python bench.py" \
  "bench_cfg3|200|python bench.py --config cfg3_resnet50_r4 --no-cpu-baseline" \
  "bw|120|tools/bw_ceiling" \
  "prof_cfg2|400|tools/profile.sh cfg2_resnet50_r1 gpurun_out/prof_cfg2 cold"
python3 tools/parity_summary.py $PSGD_PARITY_LOG > gpurun_out/parity_summary.json 2>/dev/null
exit 0
