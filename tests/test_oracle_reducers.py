"""The paper-code reducer oracle (oracle/reducers_oracle.py) against fixtures produced by
the paper code itself (tests/golden/make_golden_reducers.py): bitwise equal, every step."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import reducers_oracle as RO

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MAN = json.load(open(os.path.join(GOLDEN, "reducers_manifest.json")))


def load(name):
    with np.load(os.path.join(GOLDEN, f"R_{name}.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def draw_fn(draws):
    pos = [0]

    def fn(shape):
        n = int(np.prod(shape))
        v = torch.from_numpy(draws[pos[0]:pos[0] + n].copy()).view(shape)
        pos[0] += n
        return v

    return fn


def make_state(name, draws):
    info = MAN["scenarios"][name]
    kw = dict(info["kwargs"])
    if info["class"] == "RankKReducer":
        return RO.RankKState(7, rank=kw["rank"], reuse_query=kw["reuse_query"], random_fn=draw_fn(draws))
    return RO.HalfRankKState(7, rank=kw["rank"], random_fn=draw_fn(draws))


@pytest.mark.parametrize("name", sorted(MAN["scenarios"]))
def test_reducer_oracle_bitwise(name):
    want = load(name)
    shapes = [tuple(s) for s in MAN["shapes"]]
    st = make_state(name, want["draws"])
    memories = [torch.zeros(s) for s in shapes]
    for t in range(MAN["steps"]):
        send = [torch.from_numpy(want[f"s{t}_in_{i}"]) for i in range(len(shapes))]
        outs = [torch.empty(s) for s in shapes]
        bits = st.reduce(send, outs, memories)
        assert bits == int(want[f"s{t}_bits"])
        for i in range(len(shapes)):
            assert torch.equal(outs[i], torch.from_numpy(want[f"s{t}_out_{i}"])), (name, t, i, "out")
            assert torch.equal(memories[i], torch.from_numpy(want[f"s{t}_mem_{i}"])), (name, t, i, "mem")
