#!/bin/bash
# SQ counters (two PMC passes) of the cold cfg2/cfg3 steps: occupancy / wait / instruction mix
# per kernel, for the next round's even-product work.
set -o pipefail
O=gpurun_out/sq; mkdir -p $O
export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM"
for c in cfg2_resnet50_r1 cfg3_resnet50_r4; do
  timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv -d $O/a_$c -o sq -- python3 bench.py --config $c --steps 20 --warmup 3 --mode cold --no-cpu-baseline > $O/a_$c.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $C2 --output-format csv -d $O/b_$c -o sq -- python3 bench.py --config $c --steps 20 --warmup 3 --mode cold --no-cpu-baseline > $O/b_$c.log 2>&1 || exit 1
  python3 tools/prof_summary.py $O/a_$c | grep psgd > $O/sq_$c.txt
  python3 tools/prof_summary.py $O/b_$c | grep psgd >> $O/sq_$c.txt
done
cat $O/sq_*.txt | grep -E "product|final|reduce" | head -60
