"""Probe the rank-16 orthonormalisation (k_orth_chol16) on one k x 16 panel: time per call,
orthonormality, and agreement with LAPACK (torch.linalg.qr on the CPU, signs included).

usage (GPU box): python tools/orth16_probe.py [k] [reps] [rank 16|32]
PSGD_ORTH_DIAG=1 skips the Householder fallback (shows whether Cholesky-QR itself succeeds).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from powersgd_amd import Config, PowerSGD

k = int(sys.argv[1]) if len(sys.argv) > 1 else 4608
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
R = int(sys.argv[3]) if len(sys.argv) > 3 else 16
dev = torch.device("cuda:0")
psgd = PowerSGD([torch.zeros(k, 512, device=dev)], Config(R, 0.1, 1, 0))
plan = psgd._powersgd._plan
stream = torch.cuda.current_stream().cuda_stream
x0 = torch.randn(k, R, generator=torch.Generator().manual_seed(5))
buf = psgd._powersgd._ps_buffer
assert buf.numel() == k * R, buf.numel()
buf.copy_(x0.reshape(-1))
plan.orthogonalize(True, buf.data_ptr(), 0, stream)
torch.cuda.synchronize()
q = buf.view(k, R).cpu()
ref = torch.linalg.qr(x0).Q
orth = float((q.t() @ q - torch.eye(R)).abs().max())
diff = float((q - ref).abs().max())
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    plan.orthogonalize(True, buf.data_ptr(), 0, stream)
e1.record()
torch.cuda.synchronize()
print(f"k={k} R={R}: |Q^TQ-I|max={orth:.2e} |Q-Q_lapack|max={diff:.2e} "
      f"us/call={e0.elapsed_time(e1) / reps * 1e3:.1f} (diag={os.environ.get('PSGD_ORTH_DIAG', '0')})")
