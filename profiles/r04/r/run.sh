#!/bin/bash
# k_lowrank_out with 4 rows per lane in flight (variant lib) vs default: W>1 timing, trace, tests
tag=${1:-r04r}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
V=powersgd_amd/_lib_v/lr4/libpsgd.so
tools/gpu_steps.sh \
  "$tag-w1|500|for k in 1 2; do for lib in default $V; do if [ \$lib = default ]; then unset PSGD_LIB_PATH; else export PSGD_LIB_PATH=\$lib; fi; python tools/w_gt1_ab.py > $o/w.json 2> $o/w.err || { tail -20 $o/w.err; exit 1; }; echo \"lib=\$lib \$(grep '^{' $o/w.json)\"; done; done" \
  "$tag-kt|200|for lib in default $V; do if [ \$lib = default ]; then unset PSGD_LIB_PATH; else export PSGD_LIB_PATH=\$lib; fi; rm -rf /tmp/ktw; rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/w_gt1_ab.py > /dev/null 2>&1 || exit 1; echo \"lib=\$lib\"; python3 tools/kt_med.py /tmp/ktw 0; done" \
  "$tag-pytest|400|PSGD_LIB_PATH=$V python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_ipc.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
true
