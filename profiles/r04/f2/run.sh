#!/bin/bash
tag=${1:-r04f2}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread -p no:cacheprovider" \
  "$tag-smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "$tag-bench|400|python bench.py --steps 100 --warmup 10 > $o/bench_default.json && cat $o/bench_default.json"
true
