#!/bin/bash
# A/B of the orthonormalisation kernels: PSGD_ORTH_DIAG=2 disables the register-resident panel.
set -o pipefail
O=${1:-gpurun_out/orth_ab}; mkdir -p $O
export TMPDIR=/tmp
for v in 0 2 0 2; do
  for c in cfg3_resnet50_r4 cfg4_llama_r2_bf16; do
    PSGD_ORTH_DIAG=$v timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/kt_${c}_$v -o kt -- \
      python3 bench.py --config $c --steps 30 --warmup 4 --mode cold --no-cpu-baseline > /dev/null 2> $O/err || { tail -5 $O/err; exit 1; }
    python3 tools/prof_summary.py $O/kt_${c}_$v | grep -E "orth|reduce" | sed "s/^/$c diag=$v /"
  done
done
