#!/bin/bash
# k_orth_chol load batches: 16 rows per thread at rank 2, 12 at rank 4 (variant lib) vs 8
tag=${1:-r04t}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
V=powersgd_amd/_lib_v/chu/libpsgd.so
tools/gpu_steps.sh \
  "$tag-kt|400|for k in 1 2; do for lib in default $V; do if [ \$lib = default ]; then unset PSGD_LIB_PATH; else export PSGD_LIB_PATH=\$lib; fi; python bench.py --config cfg4_llama_r2_bf16 --steps 100 --warmup 10 --no-cpu-baseline --no-extra --mode cold > $o/w.json || exit 1; rm -rf /tmp/ktw; rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/step_trace.py cfg4_llama_r2_bf16 16 > /dev/null 2>&1 || exit 1; echo \"lib=\$lib cfg4\"; python3 -c \"import json,sys;print(json.load(open(sys.argv[1]))['ms_per_step'])\" $o/w.json; python3 tools/kt_med.py /tmp/ktw 30; done; done" \
  "$tag-w1|400|for k in 1 2; do for lib in default $V; do if [ \$lib = default ]; then unset PSGD_LIB_PATH; else export PSGD_LIB_PATH=\$lib; fi; python tools/w_gt1_ab.py > $o/w.json 2> $o/w.err || { tail -20 $o/w.err; exit 1; }; echo \"lib=\$lib \$(grep '^{' $o/w.json)\"; done; done" \
  "$tag-w1kt|200|for lib in default $V; do if [ \$lib = default ]; then unset PSGD_LIB_PATH; else export PSGD_LIB_PATH=\$lib; fi; rm -rf /tmp/ktw; rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/w_gt1_ab.py > /dev/null 2>&1 || exit 1; echo \"lib=\$lib\"; python3 tools/kt_med.py /tmp/ktw 0; done" \
  "$tag-pytest|400|PSGD_LIB_PATH=$V python -u -m pytest tests/test_gpu_orth.py tests/test_gpu_parity.py tests/test_gpu_rccl.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
true
