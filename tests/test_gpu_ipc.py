"""One-shot all-reduce of the last factor over IPC mappings (psgd_ipc_*, PSGD_IPC_ALLREDUCE=1):
W processes on cuda:0 (gloo for the host barriers and the earlier iterations' collectives), each
mapping the others' exchange buffers with hipIpcOpenMemHandle and summing them in one kernel.
Checked against the reference's own multi-worker goldens (F2), like the collective path."""
import os
import tempfile

import pytest
import torch

from golden_io import load, manifest, scenario_inputs
from parity_log import check

pytestmark = pytest.mark.gpu
MAN = manifest()
TOL_FREE = 1e-4


def _worker(rank_id, world, key, initfile):
    os.environ["PSGD_IPC_ALLREDUCE"] = "1"
    from powersgd_amd import Config, PowerSGD

    torch.distributed.init_process_group("gloo", init_method=f"file://{initfile}", rank=rank_id, world_size=world)
    try:
        info = MAN["multi"][key]
        meta = MAN["scenarios"][info["scenario"]]
        want = load("F2_" + key)
        pre = f"rank{rank_id}_"
        dev = torch.device("cuda:0")
        shapes = [tuple(s) for s in meta["shapes"]]
        psgd = PowerSGD([torch.zeros(s, device=dev) for s in shapes],
                        Config(meta["rank"], meta["mcr"], meta["iters"], meta["start"]))
        psgd._powersgd._ps_buffer.copy_(torch.from_numpy(want[pre + "p0"]).to(dev))
        psgd._powersgd._qs_buffer.copy_(torch.from_numpy(want[pre + "q0"]).to(dev))
        res = [torch.zeros(s) for s in shapes]
        for t in range(meta["steps"]):
            inputs = scenario_inputs(meta, t, res, rank_id)
            grads = [g.to(dev) for g in inputs]
            outs = psgd.aggregate(grads)
            torch.cuda.synchronize()
            for i, g in enumerate(inputs):
                scale = max(float(g.norm()), 1e-30)
                eo = float((outs[i].cpu() - torch.from_numpy(want[f"{pre}s{t}_out_{i}"])).norm()) / scale
                er = float((grads[i].cpu() - torch.from_numpy(want[f"{pre}s{t}_res_{i}"])).norm()) / scale
                check(eo, TOL_FREE, key, rank_id, t, i, "ipc-out")
                check(er, TOL_FREE, key, rank_id, t, i, "ipc-res")
            res = [g.cpu() for g in grads]
        assert psgd._powersgd._ipc_open
        torch.distributed.barrier()
    finally:
        torch.distributed.destroy_process_group()


@pytest.mark.parametrize("key", sorted(MAN["multi"]))
def test_ipc_one_shot_allreduce_matches_reference(key):
    world = MAN["multi"][key]["world"]
    with tempfile.TemporaryDirectory() as td:
        torch.multiprocessing.spawn(_worker, args=(world, key, os.path.join(td, "init")), nprocs=world, join=True)
