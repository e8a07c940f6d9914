#!/bin/bash
# Counter passes for the rank-k product kernels at HEAD (run on the GPU box):
#   1. the list of counters this rocprofv3 offers (kept for the record);
#   2. SQ stall breakdown (WAIT_ANY / WAIT_INST_ANY / ACTIVE_INST_ANY vs WAVE_CYCLES) of the
#      cold cfg2 and cfg3 bench loops: k_even<float,1> / <float,4> and the final passes;
#   3. MFMA / VALU busy of the rank-k products at ranks 1, 4, 8, 16 (tools/rank_products.py).
# usage: tools/pmc_stalls.sh <outdir>
set -e
out=$1; mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/counters_list.txt" 2>&1 || true
STALL="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
LDS="SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
MFMA="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for cfg in cfg2_resnet50_r1 cfg3_resnet50_r4; do
  mkdir -p "$out/$cfg"
  B="bench.py --config $cfg --steps 20 --warmup 3 --mode cold --no-cpu-baseline --no-extra"
  timeout -s KILL 120 rocprofv3 --pmc $STALL --output-format csv -d "$out/$cfg/stall" -o stall -- python3 $B > "$out/$cfg/stall.log" 2>&1
  if grep -q -w SQ_INSTS_LDS "$out/counters_list.txt" && grep -q -w SQ_INSTS_VMEM_RD "$out/counters_list.txt"; then
    timeout -s KILL 120 rocprofv3 --pmc $LDS --output-format csv -d "$out/$cfg/lds" -o lds -- python3 $B > "$out/$cfg/lds.log" 2>&1 || echo "lds pass failed ($cfg)"
  fi
  python3 tools/prof_summary.py "$out/$cfg" > "$out/$cfg/summary.txt"
  [ -n "$KEEP_RAW" ] || rm -rf "$out/$cfg/stall" "$out/$cfg/lds"  # gpurun returns <= 64 MiB
  echo "$cfg done"
done
for R in 1 4 8 16; do
  mkdir -p "$out/rank$R"
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$out/rank$R/kt" -o kt -- python3 tools/rank_products.py run $R > "$out/rank$R/kt.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $MFMA --output-format csv -d "$out/rank$R/pmc" -o pmc -- python3 tools/rank_products.py run $R > "$out/rank$R/pmc.log" 2>&1
  python3 tools/rank_products.py analyze "$out/rank$R" $R > "$out/rank$R/products.jsonl"
  python3 tools/prof_summary.py "$out/rank$R" > "$out/rank$R/summary.txt"
  [ -n "$KEEP_RAW" ] || rm -rf "$out/rank$R/kt" "$out/rank$R/pmc"
  echo "rank $R done"
done
echo done
