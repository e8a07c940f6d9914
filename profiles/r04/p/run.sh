#!/bin/bash
# K-term final pass on its own ~16k-element row blocks: W>1 tests, W>1 timing, default line
tag=${1:-r04p}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-pytest|600|python -u -m pytest tests/test_gpu_final.py tests/test_gpu_rccl.py tests/test_gpu_ipc.py tests/test_gpu_parity.py tests/test_gpu_bench_multi.py tests/test_gpu_multiworker.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "$tag-w1|400|for k in 1 2 3; do python tools/w_gt1_ab.py > $o/w.json 2> $o/w.err || { tail -20 $o/w.err; exit 1; }; grep '^{' $o/w.json; done" \
  "$tag-kt|200|rm -rf /tmp/ktw; rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/w_gt1_ab.py > /dev/null 2>&1 || exit 1; python3 tools/kt_med.py /tmp/ktw 0" \
  "$tag-bench|300|python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $o/b.json && python3 -c \"import json;d=json.load(open('$o/b.json'));print(d['ms_per_step'], d['roofline']['frac'], d['rank4']['ms_per_step'], d['w_gt1_path']['cfg2_resnet50_r1']['ms_per_step'], d['w_gt1_path']['cfg3_resnet50_r4']['ms_per_step'])\""
true
