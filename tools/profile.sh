#!/bin/bash
# rocprofv3 passes for one bench config and cache state: kernel trace + stats, then one PMC
# counter per pass (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE cannot share a pass).
# usage: tools/profile.sh <config> <outdir> [cold|warm]   (run on the GPU box)
set -e
cfg=$1; out=$2; cache=${3:-cold}; mkdir -p "$out"
export TMPDIR=/tmp
B="bench.py --config $cfg --steps 40 --warmup 4 --mode $cache --no-cpu-baseline --no-extra"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- python3 $B > "$out/kt.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- python3 $B > "$out/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- python3 $B > "$out/write.log" 2>&1
python3 tools/prof_summary.py "$out" --traffic "$cfg:$cache" > "$out/summary.txt"
