#!/bin/bash
set -o pipefail
O=gpurun_out/r02b_c8; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
O=gpurun_out/ab8 CFGS="cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16 cfg1_1024sq_r1" bash tools/r02b_ab.sh "" prev
