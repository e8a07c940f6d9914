#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/r02b_c6}; mkdir -p $O
export TMPDIR=/tmp
export PSGD_PARITY_LOG=$O/parity_errors.jsonl
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in cfg3_resnet50_r4 cfg4_llama_r2_bf16 cfg2_resnet50_r1; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c','cold',d['value'],d['ms_per_step'],'warm',d['warm']['value'],d['warm']['ms_per_step'],'fin_us',d['roofline']['avg_launch_us'],'frac',d['roofline']['frac'])"
done
PSGD_QFOLD=0 timeout -k 10 120 python bench.py --config cfg3_resnet50_r4 --no-cpu-baseline > $O/bench_cfg3_noqfold.json 2> $O/err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_cfg3_noqfold.json'));print('cfg3 QFOLD=0','cold',d['value'],d['ms_per_step'],'warm',d['warm']['ms_per_step'],'fin_us',d['roofline']['avg_launch_us'])"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt3 -o kt -- python3 bench.py --config cfg3_resnet50_r4 --steps 30 --warmup 4 --mode cold --no-cpu-baseline > /dev/null 2> $O/err || { tail -5 $O/err; exit 1; }
python3 tools/prof_summary.py $O/kt3 | grep psgd
python3 tools/kt_seq.py $O/kt3 10
