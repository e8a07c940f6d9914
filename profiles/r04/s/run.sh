#!/bin/bash
# per-launch floor of a dependent kernel chain (small plans)
tag=${1:-r04s}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-floor|120|./tools/launch_floor" \
  "$tag-kt|120|rm -rf /tmp/ktf; rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ktf -o kt -- ./tools/launch_floor > /dev/null && cat /tmp/ktf/*/kt_kernel_stats.csv"
true
