#!/bin/bash
# GPU suite, default bench line (with the rank-4 and world-size>1-path blocks), traces of the
# W=1 steps and of the W>1 path (1-rank RCCL group) for cfg3 / cfg2.
tag=${1:-r03}
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "$tag-pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "$tag-bench|400|python bench.py --steps 50 --warmup 10" \
  "$tag-kt3|200|rocprofv3 --kernel-trace --output-format csv -d /tmp/$tag-kt3 -o kt -- python3 bench.py --config cfg3_resnet50_r4 --steps 20 --warmup 4 --mode cold --no-cpu-baseline --no-extra && python3 tools/prof_summary.py /tmp/$tag-kt3 && python3 tools/kt_seq.py /tmp/$tag-kt3 12" \
  "$tag-kt2|200|rocprofv3 --kernel-trace --output-format csv -d /tmp/$tag-kt2 -o kt -- python3 bench.py --config cfg2_resnet50_r1 --steps 20 --warmup 4 --mode cold --no-cpu-baseline --no-extra && python3 tools/prof_summary.py /tmp/$tag-kt2 && python3 tools/kt_seq.py /tmp/$tag-kt2 9" \
  "$tag-ktw3|200|rocprofv3 --kernel-trace --output-format csv -d /tmp/$tag-ktw3 -o kt -- python3 tools/w_gt1_trace.py cfg3_resnet50_r4 12 && python3 tools/kt_seq.py /tmp/$tag-ktw3 60 all"
