#!/bin/bash
# SQ stall breakdown (one PMC pass) for a bench config and for the streaming ceiling tool.
# usage: tools/pmc_sq.sh <config> <outdir>   (run on the GPU box)
cfg=$1; out=$2; mkdir -p "$out"
export TMPDIR=/tmp
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/sq" -o sq -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline > "$out/sq.log" 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/sqbw" -o sqbw -- tools/bw_ceiling > "$out/sqbw.log" 2>&1 &&
python3 tools/prof_summary.py "$out" > "$out/summary.txt"
