"""The even product alone (psgd_product building block: k_even + k_reduce) over NS rotating
gradient sets (cold: NS x the plan's bytes >> 256 MB), for a single large matrix or the
ResNet-50 shapes. Run under rocprofv3 --kernel-trace. usage: python tools/even_alone.py
<single|resnet50> <rank> [steps] [sets] [mode]   (mode: read | write: after each product the
set is rewritten in place, as the final pass writes the residual | step: plus the output slab
write of a final pass, 2x the set)"""
import sys

import torch

sys.path.insert(0, ".")
from powersgd_amd import _lib  # noqa: E402
from powersgd_amd.workloads import resnet50_shapes  # noqa: E402

which, rank = sys.argv[1], int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 24
shapes = [(5547, 4608)] if which == "single" else [s for s in resnet50_shapes() if len(s) > 1]
dev = torch.device("cuda:0")
plan = _lib.Plan(shapes, rank, 2, _lib.PSGD_F32)
pn, qn = plan.factor_numel()
P = torch.randn(pn, device=dev)
Q = torch.zeros(qn, device=dev)
ws = torch.empty(plan.workspace_bytes(), dtype=torch.uint8, device=dev)
plan.bind(0, P.data_ptr(), Q.data_ptr(), ws.data_ptr())
nbytes = sum(torch.Size(s).numel() for s in shapes) * 4
NS = int(sys.argv[4]) if len(sys.argv) > 4 else max(4, int(1.2e9 // nbytes))
mode = sys.argv[5] if len(sys.argv) > 5 else "read"
sets = [[torch.randn(s, device=dev) for s in shapes] for _ in range(NS)]
tabs = [_lib.ptr_array([g.data_ptr() for g in st]) for st in sets]
stream = torch.cuda.current_stream().cuda_stream
outs = [torch.empty(s, device=dev) for s in shapes]
for k in range(steps):
    plan.product(tabs[k % NS], False, P.data_ptr(), Q.data_ptr(), (), stream)
    if mode in ("write", "step"):
        for g in sets[k % NS]:
            g.mul_(1.0)  # read + write the set back (the residual write of a final pass)
    if mode == "step":
        for g, o in zip(sets[k % NS], outs):
            o.copy_(g)  # one more write stream (the output)
torch.cuda.synchronize()
print(which, rank, "sets", NS, "done")
