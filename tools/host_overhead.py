"""Diagnose host overhead: time inside PowerSGD.aggregate() per call (no sync) vs the
device step time, and the C-ABI-only loop (psgd_aggregate on fixed buffers)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from powersgd_amd import Config, PowerSGD
from powersgd_amd import _lib
from powersgd_amd.workloads import CONFIGS

cfg = sys.argv[1] if len(sys.argv) > 1 else "cfg2_resnet50_r1"
c = CONFIGS[cfg]
dev = torch.device("cuda:0")
grads = [torch.randn(s, device=dev) for s in c["shapes"]]
psgd = PowerSGD([torch.zeros(s, device=dev) for s in c["shapes"]], Config(c["rank"], c["mcr"], c["iters"], 0))
for _ in range(5):
    psgd.aggregate(grads)
torch.cuda.synchronize()
K = 200
inside = 0.0
t0 = time.perf_counter()
for _ in range(K):
    a = time.perf_counter()
    psgd.aggregate(grads)
    inside += time.perf_counter() - a
torch.cuda.synchronize()
wall = time.perf_counter() - t0
print(f"{cfg}: PowerSGD.aggregate wall {wall/K*1e6:.1f} us/step, host inside call {inside/K*1e6:.1f} us/call")

codec = psgd._powersgd
comp = [g for g, m in zip(grads, psgd.is_compressed_mask) if m]
codec._table.fill(comp); ptrs = codec._table.comp_addr()
out = torch.empty(codec._out_numel, device=dev)
stream = torch.cuda.current_stream().cuda_stream
torch.cuda.synchronize()
t0 = time.perf_counter()
inside = 0.0
for k in range(K):
    a = time.perf_counter()
    codec._plan.aggregate(ptrs, out.data_ptr(), k, stream)
    inside += time.perf_counter() - a
torch.cuda.synchronize()
wall = time.perf_counter() - t0
print(f"{cfg}: psgd_aggregate (C ABI only) wall {wall/K*1e6:.1f} us/step, host inside {inside/K*1e6:.1f} us/call")
unc = [g for g, m in zip(grads, psgd.is_compressed_mask) if not m]
ar = psgd._allreduce
torch.cuda.synchronize()
t0 = time.perf_counter()
for k in range(K):
    ar.aggregate(unc)
torch.cuda.synchronize()
print(f"{cfg}: AllReduce.aggregate(uncompressed) {((time.perf_counter()-t0)/K)*1e6:.1f} us/call")
