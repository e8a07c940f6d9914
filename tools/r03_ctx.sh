#!/bin/bash
# k_even duration with and without a GPU idle spin before each step (tools/even_context.py)
out=$1; mkdir -p $out; export TMPDIR=/tmp
for cfg in cfg2_resnet50_r1 cfg3_resnet50_r4; do
  for cyc in 0 200000; do
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/kt_${cfg}_$cyc -o kt -- python3 tools/even_context.py $cfg $cyc 24 > /dev/null 2>&1 || exit 1
    python3 tools/kt_quick.py $out/kt_${cfg}_$cyc psgd | sed "s/^/$cfg sleep=$cyc /"
  done
done
