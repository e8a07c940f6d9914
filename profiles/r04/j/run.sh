#!/bin/bash
# k_even geometry at rank 4 under the cost model: workgroups per CU, segment cost
tag=${1:-r04j}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-even|600|for c in cfg3_resnet50_r4 cfg2_resnet50_r1; do for spec in 'PSGD_EVEN_WPC=4' 'PSGD_EVEN_WPC=2' 'PSGD_EVEN_WPC=3' 'PSGD_EVEN_SEGC=8192' 'PSGD_EVEN_SEGC=16384' 'PSGD_EVEN_WPC=4'; do env \$spec python bench.py --config \$c --steps 100 --warmup 10 --no-cpu-baseline --no-extra --mode cold > $o/w.json || exit 1; rm -rf /tmp/ktw; env \$spec rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/step_trace.py \$c 16 > /dev/null 2>&1 || exit 1; python3 -c \"import json;d=json.load(open('$o/w.json'));print('\$c \$spec', d['ms_per_step'], end='  ')\"; python3 tools/kt_med.py /tmp/ktw 30; done; done"
true
