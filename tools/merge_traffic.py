"""Fold gpurun_out/pmc_traffic.json (written on the GPU box by tools/prof_summary.py --traffic)
into the committed profiles/pmc_traffic.json that bench.py reads for roofline.traffic."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "pmc_traffic.json")
dst = os.path.join(REPO, "profiles", "pmc_traffic.json")
new = json.load(open(src))
try:
    cur = json.load(open(dst))
except (OSError, ValueError):
    cur = {}
cur.update(new)
json.dump(cur, open(dst, "w"), indent=1, sort_keys=True)
print(json.dumps(cur, indent=1, sort_keys=True))
