#!/bin/bash
set -o pipefail
PSGD_PROJ_S5=1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "final or parity or qfold or orth" > gpurun_out/c11_pytest.log 2>&1 || { tail -30 gpurun_out/c11_pytest.log; exit 1; }
tail -1 gpurun_out/c11_pytest.log
export TMPDIR=/tmp
O=gpurun_out/s5; mkdir -p $O
for rep in 1 2 3; do for v in 0 1; do c=cfg3_resnet50_r4
  d=$O/s5_${v}_$rep
  PSGD_PROJ_S5=$v timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- python3 bench.py --config $c --steps 30 --warmup 4 --mode cold --no-cpu-baseline > $d.json 2> $d.err || { tail -5 $d.err; exit 1; }
  echo "s5=$v ms=$(python3 -c "import json;print(json.load(open('$d.json'))['ms_per_step'])") $(python3 tools/prof_summary.py $d | grep -E 'k_final_proj' | awk '{printf "%s %s | ", $1" "$2, $(NF-2)}')"
done; done
for v in 0 1; do PSGD_PROJ_S5=$v timeout -k 10 90 python bench.py --config cfg3_resnet50_r4 --no-cpu-baseline > $O/b$v.json 2>/dev/null || exit 1; echo "s5=$v bench $(python3 -c "import json;d=json.load(open('$O/b$v.json'));print(d['ms_per_step'],d['warm']['ms_per_step'],d['roofline']['avg_launch_us'])")"; done
