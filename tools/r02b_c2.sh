#!/bin/bash
# reduce A/B (per-item widths) + SQ stall counters of the final passes (cfg2 rank 1 vs cfg3 rank 4)
set -o pipefail
O=${1:-gpurun_out/r02b_c2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "reduce or parity or golden or kernels or final or orth or multiworker or baseline" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg2_resnet50_r1 cfg3_resnet50_r4; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c','cold',d['value'],d['ms_per_step'],'warm',d['warm']['value'],d['warm']['ms_per_step'],'fin_us',d['roofline']['avg_launch_us'],'frac',d['roofline']['frac'])"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$c -o kt -- \
    python3 bench.py --config $c --steps 30 --warmup 4 --mode cold --no-cpu-baseline > /dev/null 2> $O/err || { tail -5 $O/err; exit 1; }
  python3 tools/prof_summary.py $O/kt_$c | grep psgd | head -8
done
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
for c in cfg2_resnet50_r1 cfg3_resnet50_r4; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/sq_$c -o sq -- python3 bench.py --config $c --steps 20 --warmup 3 --mode cold --no-cpu-baseline > $O/sq_$c.log 2>&1 || exit 1
  python3 tools/prof_summary.py $O/sq_$c | grep -E "final|product" > $O/sq_$c.txt
done
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM"
for c in cfg2_resnet50_r1 cfg3_resnet50_r4; do
  timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv -d $O/sq2_$c -o sq -- python3 bench.py --config $c --steps 20 --warmup 3 --mode cold --no-cpu-baseline > $O/sq2_$c.log 2>&1 || { echo sq2 failed; break; }
  python3 tools/prof_summary.py $O/sq2_$c | grep -E "final|product" >> $O/sq_$c.txt
done
cat $O/sq_*.txt
