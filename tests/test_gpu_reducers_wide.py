"""The paper-code reducers (powersgd_amd/reducers.py) at ranks 16 and 32, where psgd_reconstruct
takes the matrix-core apply tiles with separate residual / output destinations and two factor
sets (psgd_stream.cuh apply_tile_mfma), against the paper-code oracle (oracle/reducers_oracle.py,
bitwise equal to the paper code on its own fixtures: tests/test_oracle_reducers.py) on the same
inputs and the same injected query draws. The fixtures of tests/test_gpu_reducers.py stop at
rank 4; these shapes include a matrix with m % 4 != 0 (the VALU fallback) and a 1-D tensor.
Tolerance relative to the input norm: 1e-5 at the first step, 1e-4 after (as that test)."""
import numpy as np
import pytest
import torch

from oracle import reducers_oracle as RO
from powersgd_amd.reducers import HalfRankKReducer, RankKReducer

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
SHAPES = [(128, 64, 3, 3), (256, 300), (40,), (96, 200), (64, 100), (50, 150)]
STEPS = 3


def _draws(dev):
    draws = np.random.RandomState(11).standard_normal(1 << 20).astype(np.float32)
    pos = [0]

    def fn(shape):
        n = int(np.prod(shape))
        v = torch.from_numpy(draws[pos[0]:pos[0] + n].copy()).view(shape)
        pos[0] += n
        return v.to(dev) if dev is not None else v

    return fn


@pytest.mark.parametrize("cls", ["rankk", "rankk_noreuse", "halfrankk"])
@pytest.mark.parametrize("rank", [16, 32])
def test_paper_reducers_wide_ranks_vs_oracle(cls, rank):
    if cls == "halfrankk":
        red = HalfRankKReducer(7, DEV, rank=rank, random_fn=_draws(DEV))
        ora = RO.HalfRankKState(7, rank=rank, random_fn=_draws(None))
    else:
        reuse = cls == "rankk"
        red = RankKReducer(7, DEV, rank=rank, reuse_query=reuse, random_fn=_draws(DEV))
        ora = RO.RankKState(7, rank=rank, reuse_query=reuse, random_fn=_draws(None))
    g = torch.Generator().manual_seed(rank)
    mem_d = [torch.zeros(s, device=DEV) for s in SHAPES]
    mem_c = [torch.zeros(s) for s in SHAPES]
    for t in range(STEPS):
        grads = [torch.randn(s, generator=g) for s in SHAPES]
        send_c = [gr + m for gr, m in zip(grads, mem_c)]
        send_d = [gr.to(DEV) + m for gr, m in zip(grads, mem_d)]
        scale = [x.clone() for x in send_c]
        out_d = [torch.empty(s, device=DEV) for s in SHAPES]
        out_c = [torch.empty(s) for s in SHAPES]
        bits_d = red.reduce(send_d, out_d, mem_d)
        bits_c = ora.reduce(send_c, out_c, mem_c)
        torch.cuda.synchronize()
        assert bits_d == bits_c
        tol = 1e-5 if t == 0 else 1e-4
        for i in range(len(SHAPES)):
            s = max(float(scale[i].norm()), 1e-30)
            eo = float((out_d[i].cpu() - out_c[i]).norm()) / s
            em = float((mem_d[i].cpu() - mem_c[i]).norm()) / s
            assert eo <= tol and em <= tol, (cls, rank, t, i, SHAPES[i], eo, em)
        # continue each side from its own state (the memories), as the paper's training loop does
