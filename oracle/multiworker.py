"""TEST INFRASTRUCTURE ONLY — W reference workers in ONE process, for checking the multi-GPU path.

The reference's multi-worker step (powersgd/powersgd.py:204-219, utils.py:43-47) needs the SUM
of every worker's out-factor after each power iteration, so W oracle workers cannot run one
after another. Here each worker is a thread running ``powersgd_oracle.policy_step`` and the
all-reduce hook meets the others at a barrier: every worker deposits its buffer, worker 0 sums
them in rank order, every worker copies the sum back. Rank-order summation differs from a ring
all-reduce only in rounding (for W = 2 it is bitwise the same, a + b == b + a).

Used by tests/ (checked against the reference's own gloo goldens F2) and by bench.py's
multi-GPU parity check (rank 0, after every timed region). Never imported by the product.
"""
from __future__ import annotations

import threading
from typing import List, Sequence

import torch

from . import powersgd_oracle as O


def run_workers(states: Sequence[O.PolicyState], grads: Sequence[List[torch.Tensor]],
                timeout: float = 600.0) -> List[List[torch.Tensor]]:
    """One ``policy_step`` of every worker w on ``grads[w]`` (mutated into the residual, as in
    the reference); returns the outputs per worker. ``states[w]`` are advanced in place."""
    world = len(states)
    if len(grads) != world:
        raise ValueError("one gradient list per worker")
    barrier = threading.Barrier(world, timeout=timeout)
    slots: List[torch.Tensor] = [None] * world  # type: ignore[list-item]
    total: List[torch.Tensor] = [None]  # type: ignore[list-item]

    def hook(rank: int):
        def allreduce(buf: torch.Tensor) -> None:  # in-place SUM over the workers (rank order)
            slots[rank] = buf
            barrier.wait()
            if rank == 0:
                acc = slots[0].clone()
                for w in range(1, world):
                    acc += slots[w]
                total[0] = acc
            barrier.wait()
            buf.copy_(total[0])
            barrier.wait()  # nobody deposits the next buffer before every copy is done

        return allreduce

    outs: List[List[torch.Tensor]] = [None] * world  # type: ignore[list-item]
    errors: List[BaseException] = []

    def work(rank: int) -> None:
        try:
            outs[rank] = O.policy_step(states[rank], grads[rank], world, hook(rank) if world > 1 else None)
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errors.append(e)
            barrier.abort()

    threads = [threading.Thread(target=work, args=(w,)) for w in range(world)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        real = [e for e in errors if not isinstance(e, threading.BrokenBarrierError)]
        raise (real or errors)[0]
    return outs
