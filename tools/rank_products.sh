export TMPDIR=/tmp
set -e
mkdir -p gpurun_out/RP
for R in 1 2 4 8 16; do
  timeout -k 10 120 python3 tools/rank_products.py run $R >> gpurun_out/RP/steps.jsonl 2>/dev/null
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/RP/r$R -o kt -- python3 tools/rank_products.py run $R > gpurun_out/RP/r$R.log 2>&1
  python3 tools/rank_products.py analyze gpurun_out/RP/r$R $R >> gpurun_out/RP/products.jsonl
done
for R in 8 16; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/RP/pmc$R -o pmc -- python3 tools/rank_products.py run $R > gpurun_out/RP/pmc$R.log 2>&1
  python3 tools/prof_summary.py gpurun_out/RP/pmc$R > gpurun_out/RP/pmc$R.txt
done
