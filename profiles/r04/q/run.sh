#!/bin/bash
# write-only ceiling (k_lowrank_out's mix) and the W>1 path under other streaming tile sizes
tag=${1:-r04q}
export TMPDIR=/tmp
o=gpurun_out/$tag; mkdir -p $o
tools/gpu_steps.sh \
  "$tag-bw|120|./tools/bw_write" \
  "$tag-tiles|500|for k in 1 2; do for te in 0 16384 32768 4096; do if [ \$te = 0 ]; then unset PSGD_TILE_ELEMS; else export PSGD_TILE_ELEMS=\$te; fi; python tools/w_gt1_ab.py > $o/w.json 2> $o/w.err || { tail -20 $o/w.err; exit 1; }; echo \"tile_elems=\$te \$(grep '^{' $o/w.json)\"; done; done" \
  "$tag-kt|200|for te in 16384 32768; do rm -rf /tmp/ktw; PSGD_TILE_ELEMS=\$te rocprofv3 --kernel-trace --output-format csv -d /tmp/ktw -o kt -- python3 tools/w_gt1_ab.py > /dev/null 2>&1 || exit 1; echo \"tile_elems=\$te\"; python3 tools/kt_med.py /tmp/ktw 0; done"
true
