#!/bin/bash
# W>1 path: store policies, K-term final block size; rank-1 joint norm in one round trip
tag=${1:-r04o}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-pytest|400|python -u -m pytest tests/test_gpu_orth.py tests/test_gpu_rccl.py tests/test_gpu_ipc.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "$tag-w1|700|for k in 1 2; do for spec in PSGD_APPLY_NT=1 PSGD_APPLY_NT=0 PSGD_FIN_ELEMS=16640 PSGD_OUT_NT_MB=100000; do env \$spec python tools/w_gt1_ab.py > $o/w.json 2> $o/w.err || { tail -20 $o/w.err; exit 1; }; echo \"\$spec \$(cat $o/w.json)\"; done; done" \
  "$tag-kt|200|rm -rf /tmp/ktw; rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/w_gt1_ab.py > /dev/null 2>&1 || exit 1; python3 tools/kt_med.py /tmp/ktw 0"
true
