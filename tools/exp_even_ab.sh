#!/bin/bash
# even product A/B over library variants (PSGD_LIB_PATH), cold rotation, in isolation
export TMPDIR=/tmp
O=gpurun_out/evab; mkdir -p $O
for v in "$@"; do
  lib=$PWD/powersgd_amd/_lib${v:+_$v}/libpsgd.so
  for spec in "cfg3_resnet50_r4" "5120x4608:4" "cfg2_resnet50_r1"; do
    d=$O/${v:-default}_${spec//[:x]/_}
    PSGD_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o kt -- python3 tools/exp_even.py $spec even > $d.log 2>&1 || exit 1
    echo "== ${v:-default} $spec $(python3 tools/prof_summary.py $d | grep k_product | awk '{print $(NF-2)}')"
  done
done
