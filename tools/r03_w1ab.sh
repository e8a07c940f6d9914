#!/bin/bash
# A/B of the world-size > 1 path: tests of the RCCL path, then plain vs PSGD_FUSE_FINAL=2
set -o pipefail
mkdir -p gpurun_out/r03k
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_rccl.py \
  > gpurun_out/r03k/rccl.log 2>&1 || { tail -30 gpurun_out/r03k/rccl.log; exit 1; }
tail -3 gpurun_out/r03k/rccl.log
for spec in "base:" "fuse2:PSGD_FUSE_FINAL=2" "base2:" "fuse2b:PSGD_FUSE_FINAL=2"; do
  name=${spec%%:*}; envs=${spec#*:}
  ( [ -n "$envs" ] && export $envs; timeout -k 10 180 python -u tools/w_gt1_ab.py 2>gpurun_out/r03k/$name.err ) \
    > gpurun_out/r03k/$name.json || { tail gpurun_out/r03k/$name.err; exit 1; }
  echo "$name $(cat gpurun_out/r03k/$name.json)"
done
