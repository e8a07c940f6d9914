#!/bin/bash
# closing evidence at HEAD: GPU suite, smoke, default bench line (CPU baseline included), every
# BASELINE config's line, PMC traffic + traces of cfg2/cfg3 (cold), plain-step kernel sequences
tag=${1:-r04w}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-pytest|900|python -u -m pytest tests -m gpu -x -q --timeout 420 --timeout-method thread -p no:cacheprovider" \
  "$tag-smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "$tag-bench|400|python bench.py --steps 100 --warmup 10 > $o/bench_default.json && cat $o/bench_default.json" \
  "$tag-configs|500|for c in cfg1_1024sq_r1 cfg4_llama_r2_bf16 cfg5_lstm_r1_i4 cfg3_resnet50_r4; do python bench.py --config \$c --steps 100 --warmup 10 --no-cpu-baseline --no-extra > $o/bench_\$c.json || exit 1; python3 -c \"import json;d=json.load(open('$o/bench_'+'\$c'+'.json'));print('\$c', d['value'], d['ms_per_step'], d['roofline']['kernel'][:24], d['roofline']['frac'], 'warm', d['warm']['ms_per_step'], 'post_backward', d['post_backward']['ms_per_step'])\"; done" \
  "$tag-prof2|300|bash tools/profile.sh cfg2_resnet50_r1 $o/cfg2 cold && cat $o/cfg2/summary.txt" \
  "$tag-prof3|300|bash tools/profile.sh cfg3_resnet50_r4 $o/cfg3 cold && cat $o/cfg3/summary.txt && cp profiles/pmc_traffic.json $o/" \
  "$tag-kt|300|for c in cfg2_resnet50_r1 cfg3_resnet50_r4 cfg1_1024sq_r1 cfg4_llama_r2_bf16 cfg5_lstm_r1_i4; do rm -rf /tmp/ktz; rocprofv3 --kernel-trace --output-format csv -d /tmp/ktz -o kt -- python3 tools/step_trace.py \$c 16 > /dev/null 2>&1 || exit 1; echo \"## \$c\"; python3 tools/kt_seq.py /tmp/ktz 12; python3 tools/kt_med.py /tmp/ktz 40; done" \
  "$tag-w1kt|200|rm -rf /tmp/ktw; rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/w_gt1_ab.py > $o/w1.json 2>/dev/null || exit 1; cat $o/w1.json; python3 tools/kt_med.py /tmp/ktw 0"
rm -rf $o/cfg2/kt $o/cfg2/fetch $o/cfg2/write $o/cfg3/kt $o/cfg3/fetch $o/cfg3/write 2>/dev/null
true
