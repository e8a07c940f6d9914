#!/bin/bash
# rocprofv3 passes for one bench config: kernel trace + stats, then one PMC counter per pass.
# usage: tools/profile.sh <config> <outdir>   (run on the GPU box)
set -e
cfg=$1; out=$2; mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- python3 $B > "$out/kt.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- python3 $B > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- python3 $B > "$out/write.log" 2>&1
python3 tools/prof_summary.py "$out" --traffic "$cfg" > "$out/summary.txt"
