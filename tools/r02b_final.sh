#!/bin/bash
# round-2 closing measurements (second session): GPU suite (+ parity log), smoke, default bench,
# every config, cold kernel traces + PMC traffic for cfg2 and cfg3. Output under gpurun_out/final2/.
set -o pipefail
O=${OUT:-gpurun_out/final2}; mkdir -p $O
export PSGD_PARITY_LOG=$O/parity_errors.jsonl
rm -f $PSGD_PARITY_LOG
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
python3 tools/parity_summary.py $PSGD_PARITY_LOG > $O/parity_summary.json
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_default.json'));print('default',d['value'],d['ms_per_step'],'frac',d['roofline']['frac'],'cpu',d['cpu_baseline']['value'])"
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c','cold',d['value'],d['ms_per_step'],'warm',d['warm']['value'],d['warm']['ms_per_step'],'frac',d['roofline']['frac'],d['roofline']['kernel'][:14])"
done
PSGD_FIN_PRODUCT=1 timeout -k 10 120 python bench.py --config cfg5_lstm_r1_i4 --no-cpu-baseline > $O/bench_cfg5_finprod.json 2> $O/err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_cfg5_finprod.json'));print('cfg5 FIN_PRODUCT=1','cold',d['ms_per_step'],'warm',d['warm']['ms_per_step'])"
bash tools/profile.sh cfg2_resnet50_r1 $O/prof_cfg2 cold || exit 1
bash tools/profile.sh cfg3_resnet50_r4 $O/prof_cfg3 cold || exit 1
grep -E "psgd|traffic" $O/prof_cfg2/summary.txt | head -12
grep -E "psgd|traffic" $O/prof_cfg3/summary.txt | head -14
