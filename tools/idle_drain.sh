#!/bin/bash
# k_even after an idle gap and/or an L2 write-back: plain cold steps with 0 / 30 us of GPU idle spin
# between them (PSGD_TRACE_IDLE_US) and with or without a system-fence event after each step
# (PSGD_TRACE_FLUSH), tools/step_trace.py; kernel medians and step period per setting. GPU box.
set -e
mkdir -p gpurun_out/r06g; export TMPDIR=/tmp
for flush in 0 1; do
for idle in 0 30; do
  for cfg in cfg2_resnet50_r1 cfg3_resnet50_r4; do
    d=gpurun_out/r06g/idle$idle.flush$flush.$cfg
    PSGD_TRACE_FLUSH=$flush PSGD_TRACE_IDLE_US=$idle timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 tools/step_trace.py $cfg 60 > $d.log 2>&1
    echo "flush=$flush idle=$idle $cfg: $(python3 tools/kt_steps.py $d 150)" | tee -a gpurun_out/r06g/summary.txt
    rm -rf $d
  done
done
done
