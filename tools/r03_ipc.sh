#!/bin/bash
# IPC exchange (psgd_aggregate_ipc) on the GPU: its tests, the multi-worker / RCCL tests, the
# default bench line (W>1-path blocks incl. the exchange at W = 1) and a trace of the exchange path.
tag=${1:-r03ipc}
export TMPDIR=/tmp
tools/gpu_steps.sh \
  "$tag-pytest|600|python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_rccl.py tests/test_gpu_multiworker.py -x -v --timeout 200 --timeout-method thread" \
  "$tag-bench|400|python bench.py --steps 50 --warmup 10 --no-cpu-baseline" \
  "$tag-ktx|200|PSGD_COMM=ipc rocprofv3 --kernel-trace --output-format csv -d /tmp/$tag-ktx -o kt -- python3 tools/w_gt1_trace.py cfg3_resnet50_r4 12 && python3 tools/kt_seq.py /tmp/$tag-ktx 30 all"
