#!/bin/bash
set -o pipefail
O=${1:-gpurun_out/r02b_c4}; mkdir -p $O
export TMPDIR=/tmp
for k in 4608 2048 512; do timeout -k 5 30 tools/chol_stamps $k 54 || exit 1; done
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "orth or sign or final or parity or proj or edges" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in cfg3_resnet50_r4 cfg4_llama_r2_bf16 cfg2_resnet50_r1; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c','cold',d['value'],d['ms_per_step'],'warm',d['warm']['value'],d['warm']['ms_per_step'],'fin_us',d['roofline']['avg_launch_us'],'frac',d['roofline']['frac'])"
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt3 -o kt -- python3 bench.py --config cfg3_resnet50_r4 --steps 30 --warmup 4 --mode cold --no-cpu-baseline > /dev/null 2> $O/err || { tail -5 $O/err; exit 1; }
python3 tools/prof_summary.py $O/kt3 | grep psgd
