#!/bin/bash
# GPU suite + per-config cold bench lines and kernel traces (round 2, second session).
# usage (GPU box): bash tools/r02b_check.sh <outdir> [pytest args...]
set -o pipefail
O=${1:-gpurun_out/r02b_check}; shift; mkdir -p $O
export PSGD_PARITY_LOG=$O/parity_errors.jsonl
rm -f $PSGD_PARITY_LOG
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c','cold',d['value'],d['ms_per_step'],'warm',d['warm']['value'],d['warm']['ms_per_step'],'fin_us',d['roofline']['avg_launch_us'],'frac',d['roofline']['frac'])"
done
bash tools/r02b_base.sh $O/kt > /dev/null || exit 1
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
  echo "== $c"; grep psgd $O/kt/sum_$c.txt | head -8
done
