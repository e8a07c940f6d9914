#!/bin/bash
# Closing measurement set of a round (GPU box): GPU suite, smoke, default bench line, rocprofv3
# kernel stats of the bench command, plain-step kernel medians per config, PMC traffic of the
# final passes. Raw rocprofv3 CSVs are summarised and deleted (gpurun returns <= 64 MiB).
# usage: tools/fin_set.sh <outdir>
out=$1; mkdir -p "$out"; export TMPDIR=/tmp
step() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "=== $name"; timeout -k 10 "$secs" "$@"; local rc=$?
  echo "=== $name rc=$rc"
  case $rc in 0|1) return 0 ;; *) exit $rc ;; esac
}
step pytest 900 bash -c "python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; tail -3 $out/pytest.log"
step smoke 300 bash -c "python -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.txt 2>&1; cat $out/smoke.txt"
step bench 400 bash -c "python bench.py > $out/bench_default.json 2> $out/bench_default.err; head -c 400 $out/bench_default.json"
step stats 400 bash -c "rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o st -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/stats.log 2>&1; python3 tools/prof_summary.py $out/stats > $out/bench_kernel_summary.txt; cp \$(find $out/stats -name '*kernel_stats.csv' | head -1) $out/bench_kernel_stats.csv; rm -rf $out/stats; head -30 $out/bench_kernel_summary.txt"
for cfg in cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16 cfg5_lstm_r1_i4; do
  step "kt_$cfg" 200 bash -c "rocprofv3 --kernel-trace --output-format csv -d $out/kt_$cfg -o kt -- python3 tools/step_trace.py $cfg 60 > $out/kt_$cfg.log 2>&1; echo \"$cfg: \$(python3 tools/kt_steps.py $out/kt_$cfg 150)\" >> $out/kt_med.txt; rm -rf $out/kt_$cfg; tail -1 $out/kt_med.txt"
done
for cfg in cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
  step "pmc_$cfg" 600 bash -c "PSGD_TRAFFIC_OUT=$out/pmc_traffic.json bash tools/profile.sh $cfg $out/pmc_$cfg cold; rm -rf $out/pmc_$cfg/kt $out/pmc_$cfg/fetch $out/pmc_$cfg/write; tail -2 $out/pmc_$cfg/summary.txt"
done
echo "=== done"
