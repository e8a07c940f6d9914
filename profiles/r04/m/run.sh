#!/bin/bash
# k_apply store policy (nt vs write-through) on cfg4 and the W>1 path; K-term final block size
tag=${1:-r04m}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-cfg4|300|for k in 1 2; do for an in 1 0; do PSGD_APPLY_NT=\$an python bench.py --config cfg4_llama_r2_bf16 --steps 100 --warmup 10 --no-cpu-baseline --no-extra > $o/w.json || exit 1; rm -rf /tmp/ktw; PSGD_APPLY_NT=\$an rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/step_trace.py cfg4_llama_r2_bf16 16 > /dev/null 2>&1 || exit 1; python3 -c \"import json;d=json.load(open('$o/w.json'));print('apply_nt=\$an', d['ms_per_step'], d.get('warm',{}).get('ms_per_step'), d.get('post_backward',{}).get('ms_per_step'), end='  ')\"; python3 tools/kt_med.py /tmp/ktw 30; done; done" \
  "$tag-w1|600|for k in 1 2; do for spec in PSGD_APPLY_NT=1 PSGD_APPLY_NT=0 PSGD_FIN_ELEMS=16640 PSGD_OUT_NT_MB=100000; do env \$spec python tools/w_gt1_ab.py > $o/w.json 2> $o/w.err || { tail -20 $o/w.err; exit 1; }; echo \"\$spec \$(cat $o/w.json)\"; done; done"
true
