#!/bin/bash
# Ranks 8 / 16 / 32 at ResNet-50 shapes (GPU box): kernel-trace medians and the MFMA / VALU busy
# pass of the rank-k product kernels (tools/rank_products.py), after an optional pytest selection.
# usage: [VARIANTS="v1 v2"] tools/rank_wide.sh <outdir> "<ranks>" [pytest args...]
set -e
out=$1; ranks=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > "$out/pytest.log" 2>&1
  tail -3 "$out/pytest.log"
fi
MFMA="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
for R in $ranks; do
  # library variants (powersgd_amd/_lib_v/<name>, tools/build_variant.sh): kernel trace only
  for v in $VARIANTS; do
    d="$out/$v.rank$R"; mkdir -p "$d"
    PSGD_LIB_PATH=$PWD/powersgd_amd/_lib_v/$v/libpsgd.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv \
      -d "$d/kt" -o kt -- python3 tools/rank_products.py run $R > "$d/kt.log" 2>&1
    python3 tools/rank_products.py analyze "$d" $R > "$d/products.jsonl"; rm -rf "$d/kt"
    echo "variant $v rank $R"; cat "$d/products.jsonl"; grep ms_per_step "$d/kt.log" || true
  done
  mkdir -p "$out/rank$R"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/rank$R/kt" -o kt -- python3 tools/rank_products.py run $R > "$out/rank$R/kt.log" 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $MFMA --output-format csv -d "$out/rank$R/pmc" -o pmc -- python3 tools/rank_products.py run $R > "$out/rank$R/pmc.log" 2>&1
  python3 tools/rank_products.py analyze "$out/rank$R" $R > "$out/rank$R/products.jsonl"
  python3 tools/prof_summary.py "$out/rank$R" > "$out/rank$R/summary.txt"
  [ -n "$KEEP_RAW" ] || rm -rf "$out/rank$R/kt" "$out/rank$R/pmc"
  echo "rank $R"; cat "$out/rank$R/products.jsonl"; grep ms_per_step "$out/rank$R/kt.log" || true
done
echo done
