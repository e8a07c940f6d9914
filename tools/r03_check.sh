#!/bin/bash
# Round-3 check on the GPU box: GPU suite, cold benches of the two ResNet-50 configs, kernel traces.
# usage: tools/r03_check.sh <tag>
tag=${1:-r03}
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "$tag-pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "$tag-bench2|240|python bench.py --config cfg2_resnet50_r1 --steps 50 --warmup 10 --no-cpu-baseline" \
  "$tag-bench3|240|python bench.py --config cfg3_resnet50_r4 --steps 50 --warmup 10 --no-cpu-baseline" \
  "$tag-kt2|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag-kt2 -o kt -- python3 bench.py --config cfg2_resnet50_r1 --steps 20 --warmup 4 --mode cold --no-cpu-baseline && python3 tools/prof_summary.py gpurun_out/$tag-kt2" \
  "$tag-kt3|300|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag-kt3 -o kt -- python3 bench.py --config cfg3_resnet50_r4 --steps 20 --warmup 4 --mode cold --no-cpu-baseline && python3 tools/prof_summary.py gpurun_out/$tag-kt3"
