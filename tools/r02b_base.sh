#!/bin/bash
# Kernel sequences (cold) of every BASELINE config at HEAD: where each step's time goes.
# usage (GPU box): bash tools/r02b_base.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/r02b}; mkdir -p $O
export TMPDIR=/tmp
for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg2_resnet50_r1 cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$c -o kt -- \
    python3 bench.py --config $c --steps 30 --warmup 4 --mode cold --no-cpu-baseline > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 tools/kt_seq.py $O/kt_$c 24 > $O/seq_$c.txt
  python3 tools/prof_summary.py $O/kt_$c > $O/sum_$c.txt
  echo "== $c"; grep psgd $O/sum_$c.txt | head -12
done
