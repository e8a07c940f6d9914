#!/bin/bash
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "parity or golden or kernels or final or qfold or multiworker or reducers or training or edges" > gpurun_out/c9_pytest.log 2>&1 || { tail -30 gpurun_out/c9_pytest.log; exit 1; }
tail -1 gpurun_out/c9_pytest.log
bash tools/exp_even_ab.sh "" prev || exit 1
O=gpurun_out/ab9 CFGS="cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16" bash tools/r02b_ab.sh "" prev
