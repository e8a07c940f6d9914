#!/bin/bash
set -e
export TMPDIR=/tmp
O=gpurun_out/even; mkdir -p $O
i=0
for spec in "cfg3_resnet50_r4 even" "5120x4608:4 even" "49152x512:4 even" "20480x1152:4 even" "5120x4608:1 even" "cfg2_resnet50_r1 even"; do
  set -- $spec
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r$i -o kt -- python3 tools/exp_even.py $1 $2 > $O/r$i.log 2>&1
  echo "== $spec"; python3 tools/prof_summary.py $O/r$i | grep "k_product"
done
