"""Per-kernel register / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

usage: python tools/regs.py <source.hip> [name-substring]   (run from powersgd_amd/csrc)
"""
import os
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
EXTRA = os.environ.get("EXTRA", "").split()
cmd = ["/opt/rocm/bin/hipcc", *EXTRA, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I../../include",
       "-x", "hip", "-c", src, "-o", "/tmp/_regs.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    txt = m.group(1).strip()
    if txt.startswith("Function Name:"):
        cur = {"name": subprocess.run(["c++filt", txt.split(":", 1)[1].strip()], capture_output=True,
                                      text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if filt in r["name"]:
        print(f"{r['name'][:70]:70s} vgpr={r.get('VGPRs'):>4s} agpr={r.get('AGPRs'):>4s} "
              f"occ={r.get('Occupancy [waves/SIMD]'):>2s} vspill={r.get('VGPRs Spill'):>4s} "
              f"sspill={r.get('SGPRs Spill'):>3s} lds={r.get('LDS Size [bytes/block]')}")
