#!/bin/bash
# final-pass row-block size around the defaults: cfg2 (~8.3k elements) and cfg3 (~16.6k)
tag=${1:-r04n}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-fin|700|for k in 1 2; do for spec in cfg2_resnet50_r1:0 cfg2_resnet50_r1:5120 cfg2_resnet50_r1:6400 cfg2_resnet50_r1:10240 cfg2_resnet50_r1:12800 cfg3_resnet50_r4:0 cfg3_resnet50_r4:12288 cfg3_resnet50_r4:24576 cfg3_resnet50_r4:32768; do c=\${spec%%:*}; fe=\${spec##*:}; if [ \$fe = 0 ]; then unset PSGD_FIN_ELEMS; else export PSGD_FIN_ELEMS=\$fe; fi; python bench.py --config \$c --steps 200 --warmup 10 --no-cpu-baseline --no-extra --mode cold > $o/w.json || exit 1; python3 -c \"import json;d=json.load(open('$o/w.json'));print('\$c fin_elems=\$fe', d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])\"; done; done"
true
