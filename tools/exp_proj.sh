#!/bin/bash
# cfg3 projection-form final pass: kernel trace, SQ counters, fin_elems sweep
set -e
export TMPDIR=/tmp
O=gpurun_out/proj
mkdir -p $O
B="bench.py --config cfg3_resnet50_r4 --steps 30 --warmup 5 --mode cold --no-cpu-baseline"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $B > $O/kt.log 2>&1
python3 tools/prof_summary.py $O/kt | head -16
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d $O/sq -o sq -- python3 $B > $O/sq.log 2>&1
python3 tools/prof_summary.py $O/sq | grep -i "final_proj\|k_apply\|k_product" | head -30
for e in 8192 12288 24576 32768; do
  PSGD_FIN_ELEMS=$e timeout -k 10 100 python3 bench.py --config cfg3_resnet50_r4 --steps 50 --no-cpu-baseline > $O/fe_$e.json
  python3 -c "import json; d=json.load(open('$O/fe_$e.json')); print('fin_elems $e', d['ms_per_step'], d['warm']['ms_per_step'], d['roofline']['avg_launch_us'])"
done
