"""The paper-code reducers on the HIP codec (powersgd_amd/reducers.py) against fixtures the
paper code produced (tests/golden/make_golden_reducers.py): same inputs every step, the
paper's own random query draws injected. Tolerance relative to the input norm: 1e-5 at the
first step, 1e-4 after (the factor state evolves from the GPU's own rounding)."""
import json
import os

import numpy as np
import pytest
import torch

from powersgd_amd.reducers import HalfRankKReducer, RankKReducer

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAN = json.load(open(os.path.join(GOLDEN, "reducers_manifest.json")))


def load(name):
    with np.load(os.path.join(GOLDEN, f"R_{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def draw_fn(draws):
    pos = [0]

    def fn(shape):
        n = int(np.prod(shape))
        v = torch.from_numpy(draws[pos[0]:pos[0] + n].copy()).view(shape).to(DEV)
        pos[0] += n
        return v

    return fn


@pytest.mark.parametrize("name", sorted(MAN["scenarios"]))
def test_paper_reducers_match_paper_code(name):
    info = MAN["scenarios"][name]
    want = load(name)
    shapes = [tuple(s) for s in MAN["shapes"]]
    kw = dict(info["kwargs"])
    if info["class"] == "RankKReducer":
        red = RankKReducer(7, DEV, rank=kw["rank"], reuse_query=kw["reuse_query"], random_fn=draw_fn(want["draws"]))
    else:
        red = HalfRankKReducer(7, DEV, rank=kw["rank"], random_fn=draw_fn(want["draws"]))
    memories = [torch.zeros(s, device=DEV) for s in shapes]
    for t in range(MAN["steps"]):
        send = [torch.from_numpy(want[f"s{t}_in_{i}"]).to(DEV) for i in range(len(shapes))]
        outs = [torch.empty(s, device=DEV) for s in shapes]
        bits = red.reduce(send, outs, memories)
        torch.cuda.synchronize()
        assert bits == int(want[f"s{t}_bits"])
        tol = 1e-5 if t == 0 else 1e-4
        for i in range(len(shapes)):
            x = torch.from_numpy(want[f"s{t}_in_{i}"])
            scale = max(float(x.norm()), 1e-30)
            eo = float((outs[i].cpu() - torch.from_numpy(want[f"s{t}_out_{i}"])).norm()) / scale
            em = float((memories[i].cpu() - torch.from_numpy(want[f"s{t}_mem_{i}"])).norm()) / scale
            assert eo <= tol and em <= tol, (name, t, i, shapes[i], eo, em)
