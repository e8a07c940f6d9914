#!/bin/bash
# rank-4 ResNet-50 with one power iteration: the fused final (K = 0) vs the unfused odd step
set -e
mkdir -p gpurun_out/r4i1
export TMPDIR=/tmp
for f in 0 2; do
  PSGD_FUSE_FINAL=$f timeout -k 10 120 python bench.py --config cfg3_resnet50_r4 --iters 1 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r4i1/b_$f.json
  python -c "import json; d=json.load(open('gpurun_out/r4i1/b_$f.json')); print('fuse=$f', d['ms_per_step'], d['warm']['ms_per_step'], d['roofline']['avg_launch_us'])"
  PSGD_FUSE_FINAL=$f timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r4i1/p$f -o run -- python bench.py --config cfg3_resnet50_r4 --iters 1 --steps 50 --warmup 5 --mode cold --no-cpu-baseline > /dev/null
done
python tools/prof_summary.py gpurun_out/r4i1/p0 2>/dev/null | head -20 || true
python tools/prof_summary.py gpurun_out/r4i1/p2 2>/dev/null | head -20 || true
