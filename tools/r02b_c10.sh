#!/bin/bash
set -o pipefail
PSGD_PROD_WAVE=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "parity or golden or kernels or final or qfold or edges or orth" > gpurun_out/c10_pytest.log 2>&1 || { tail -30 gpurun_out/c10_pytest.log; exit 1; }
tail -1 gpurun_out/c10_pytest.log
export TMPDIR=/tmp
O=gpurun_out/wave; mkdir -p $O
for rep in 1 2; do for w in 0 1; do for c in cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16 cfg5_lstm_r1_i4 cfg1_1024sq_r1; do
  d=$O/w${w}_${c}_$rep
  PSGD_PROD_WAVE=$w timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 bench.py --config $c --steps 30 --warmup 4 --mode cold --no-cpu-baseline > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
  echo "wave=$w $c ms=$(python3 -c "import json;print(json.load(open('$d.json'))['ms_per_step'])") $(python3 tools/prof_summary.py $d | grep -E 'k_product|k_reduce' | awk '{printf "%s %s | ", $1" "$2, $(NF-2)}')"
done; done; done
