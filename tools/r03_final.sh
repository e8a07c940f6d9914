#!/bin/bash
# Closing evidence at HEAD: GPU suite, smoke, the default bench line (CPU baseline included),
# every BASELINE config's cold line, PMC traffic + cold traces of cfg2/cfg3, plain-step traces.
tag=${1:-r03z}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "$tag-smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "$tag-bench|400|python bench.py --steps 100 --warmup 10 > $o/bench_default.json && cat $o/bench_default.json" \
  "$tag-configs|400|for c in cfg1_1024sq_r1 cfg4_llama_r2_bf16 cfg5_lstm_r1_i4 cfg3_resnet50_r4; do python bench.py --config \$c --steps 100 --warmup 10 --no-cpu-baseline --no-extra > $o/bench_\$c.json || exit 1; python3 -c \"import json;d=json.load(open('$o/bench_'+'\$c'+'.json'));print('\$c', d['value'], d['ms_per_step'], d['roofline']['kernel'][:24], d['roofline']['frac'])\"; done" \
  "$tag-prof2|300|bash tools/profile.sh cfg2_resnet50_r1 $o/cfg2 cold && cat $o/cfg2/summary.txt" \
  "$tag-prof3|300|bash tools/profile.sh cfg3_resnet50_r4 $o/cfg3 cold && cat $o/cfg3/summary.txt && cp profiles/pmc_traffic.json $o/" \
  "$tag-kt|200|for c in cfg2_resnet50_r1 cfg3_resnet50_r4; do rocprofv3 --kernel-trace --output-format csv -d /tmp/$tag-kt\$c -o kt -- python3 tools/step_trace.py \$c 12 > /dev/null 2>&1 && python3 tools/kt_seq.py /tmp/$tag-kt\$c 10 || exit 1; done"
rm -rf $o/cfg2/kt $o/cfg2/fetch $o/cfg2/write $o/cfg3/kt $o/cfg3/fetch $o/cfg3/write 2>/dev/null
true
