#!/bin/bash
# Grid-barrier vs kernel-boundary cost, PMC traffic + cold traces of cfg2/cfg3, the host
# end-to-end flow, and the small-plan (cfg1/cfg5) step traces.
tag=${1:-r03r}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-barrier|60|./tools/grid_barrier" \
  "$tag-prof2|300|bash tools/profile.sh cfg2_resnet50_r1 $o/cfg2 cold && cat $o/cfg2/summary.txt" \
  "$tag-prof3|300|bash tools/profile.sh cfg3_resnet50_r4 $o/cfg3 cold && cat $o/cfg3/summary.txt && cp profiles/pmc_traffic.json $o/" \
  "$tag-host|300|python3 tools/host_e2e.py cfg2_resnet50_r1 20 1,2,4,8 > $o/host_e2e_cfg2.json && python3 tools/host_e2e.py cfg3_resnet50_r4 20 1,4 > $o/host_e2e_cfg3.json && cat $o/host_e2e_cfg2.json $o/host_e2e_cfg3.json" \
  "$tag-kt15|200|for c in cfg1_1024sq_r1 cfg5_lstm_r1_i4 cfg2_resnet50_r1 cfg3_resnet50_r4; do rocprofv3 --kernel-trace --output-format csv -d /tmp/$tag-kt\$c -o kt -- python3 tools/step_trace.py \$c 12 > /dev/null 2>&1 && python3 tools/kt_seq.py /tmp/$tag-kt\$c 24 || exit 1; done"
rm -rf $o/cfg2/kt $o/cfg2/fetch $o/cfg2/write $o/cfg3/kt $o/cfg3/fetch $o/cfg3/write 2>/dev/null
true
