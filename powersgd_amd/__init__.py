"""powersgd_amd — MI355X-native PowerSGD gradient compression.

Drop-in for epfml/powersgd (``powersgd/__init__.py``): same public names.

    from powersgd_amd import PowerSGD, Config, optimizer_step

The compress/decompress hot path runs in libpsgd.so (hand-written HIP for gfx950,
C ABI in include/psgd.h); the factor all-reduce uses torch.distributed (RCCL on ROCm).
"""
import torch

from powersgd_amd.powersgd import Aggregator, AllReduce, Config, PowerSGD  # noqa: F401
from powersgd_amd.utils import params_in_optimizer

__all__ = ["Aggregator", "AllReduce", "Config", "PowerSGD", "optimizer_step"]


def optimizer_step(optimizer: torch.optim.Optimizer, aggregator: Aggregator):
    """Aggregate gradients across workers with ``aggregator``, then take an optimizer
    step with the aggregate; afterwards ``p.grad`` holds the error-feedback buffer
    (reference powersgd/__init__.py:7-25)."""
    params = params_in_optimizer(optimizer)
    grads = [p.grad.data for p in params]  # type: ignore
    avg_grads = aggregator.aggregate(grads)  # subtracts the approximation from grads
    for p, g in zip(params, avg_grads):
        p.grad = g
    optimizer.step()
    for p, g in zip(params, grads):
        p.grad = g
