"""Reduce tests/parity_log.py's JSON lines to the worst observed error per test (and per
test family), with its bound: python tools/parity_summary.py gpurun_out/parity_errors.jsonl"""
import json
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/parity_errors.jsonl"
    worst = {}
    fam = defaultdict(lambda: [0.0, None, 0])
    with open(path) as f:
        for line in f:
            r = json.loads(line)
            key = r["test"]
            if key not in worst or r["err"] > worst[key]["err"]:
                worst[key] = r
            fk = re.sub(r"\[.*\]$", "", key)
            e = fam[fk]
            e[0] = max(e[0], r["err"])
            e[1] = r["tol"] if e[1] is None else max(e[1], r["tol"])
            e[2] += 1
    out = {"per_test": {k: {"max_err": v["err"], "tol": v["tol"], "headroom": (v["tol"] / v["err"]) if v["err"] else None,
                            "where": v["ctx"]} for k, v in sorted(worst.items())},
           "per_family": {k: {"max_err": v[0], "max_tol": v[1], "comparisons": v[2]} for k, v in sorted(fam.items())}}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
