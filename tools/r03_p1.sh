#!/bin/bash
# rank-1 projection form: final-pass tests, parity, bench, cfg2 trace
tag=${1:-r03p}
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "$tag-pytest|600|python -u -m pytest tests/test_gpu_final.py tests/test_gpu_parity.py tests/test_gpu_ipc.py -x -q --timeout 200 --timeout-method thread" \
  "$tag-bench|400|python bench.py --steps 50 --warmup 10 --no-cpu-baseline" \
  "$tag-kt2|200|rocprofv3 --kernel-trace --output-format csv -d /tmp/$tag-kt2 -o kt -- python3 bench.py --config cfg2_resnet50_r1 --steps 20 --warmup 4 --mode cold --no-cpu-baseline --no-extra && python3 tools/prof_summary.py /tmp/$tag-kt2 && python3 tools/kt_seq.py /tmp/$tag-kt2 9"
