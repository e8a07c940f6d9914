"""Edge shapes through the HIP path against the CPU oracle (bit-identical to the
reference): single-row and single-column matrices, 5-D tensors, ranks above the smaller
dimension, odd widths on the scalar (non-vector) layout, and the reference's errors."""
import pytest
import torch

from oracle import powersgd_oracle as O
from powersgd_amd import Config, PowerSGD
from powersgd_amd.workloads import hash_tensors

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

EDGE = [(1, 1000), (1000, 1), (2, 3, 4, 5, 6), (5, 7), (7, 5), (33, 65), (65, 33), (1, 1), (3,), (2, 2)]


@pytest.mark.parametrize("rank,iters,mcr", [(1, 2, 0.01), (3, 1, 0.01), (2, 3, 0.5), (8, 2, 0.01)])
def test_edge_shapes_vs_oracle(rank, iters, mcr):
    psgd = PowerSGD([torch.zeros(s, device=DEV) for s in EDGE], Config(rank, mcr, iters, 0))
    ora = O.policy_init([torch.zeros(s) for s in EDGE], rank, mcr, iters, 0)
    assert psgd.is_compressed_mask == ora.mask
    ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
    ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())
    for t in range(2):
        g = [torch.from_numpy(f) for f in hash_tensors(EDGE, seed=60 + t)]
        gd = [x.to(DEV) for x in g]
        gc = [x.clone() for x in g]
        outs = psgd.aggregate(gd)
        oc = O.policy_step(ora, gc)
        torch.cuda.synchronize()
        for i, x in enumerate(g):
            scale = max(float(x.norm()), 1e-30)
            assert float((outs[i].cpu() - oc[i]).norm()) / scale <= 1e-5, (t, i, EDGE[i], "out")
            assert float((gd[i].cpu() - gc[i]).norm()) / scale <= 1e-5, (t, i, EDGE[i], "res")
        # keep both on the same state (degenerate panels make the free-running state ill-posed)
        ora.codec.p_flat.copy_(psgd._powersgd._ps_buffer.cpu())
        ora.codec.q_flat.copy_(psgd._powersgd._qs_buffer.cpu())


def test_reference_errors():
    params = [torch.zeros(8, 8, device=DEV), torch.zeros(8, device=DEV)]
    psgd = PowerSGD(params, Config(1, 0.1, 1, 0))
    with pytest.raises(RuntimeError):  # non-contiguous gradient (reference view(), :289)
        psgd.aggregate([torch.zeros(8, 16, device=DEV)[:, ::2], torch.zeros(8, device=DEV)])
    with pytest.raises(RuntimeError):  # dtype mismatch (reference bmm, :189)
        psgd.aggregate([torch.zeros(8, 8, device=DEV, dtype=torch.float64), torch.zeros(8, device=DEV)])
    with pytest.raises(IndexError):  # nothing compressible (reference :118)
        PowerSGD([torch.zeros(8, device=DEV)], Config(1, 2, 1, 0))
    with pytest.raises(ValueError):  # gradient count mismatch
        psgd.aggregate([torch.zeros(8, 8, device=DEV)])
