#!/bin/bash
# session 6: suite (+ parity log) with the folded even reduction; benches with/without it
export PSGD_PARITY_LOG=gpurun_out/parity_errors.jsonl
rm -f $PSGD_PARITY_LOG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; tail -4 gpurun_out/t.log
python3 tools/parity_summary.py $PSGD_PARITY_LOG > gpurun_out/parity_summary.json
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
  for v in "" "PSGD_FOLD=0"; do
    env $v timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
    echo "$c [$v] $(python3 -c "import json;d=json.loads([l for l in open('gpurun_out/b.log') if l.startswith('{')][0]);print('cold',d['value'],d['ms_per_step'],'warm',d['warm']['value'],d['warm']['ms_per_step'])")"
  done
done
