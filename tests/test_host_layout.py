"""CPU tests of the host side: the C ABI loads and exports every declared symbol, and the
plan's layout (groups, factor sizes, output offsets, compression policy) equals the
reference's (via the bit-identical oracle). No GPU compute here."""
import os
import re

import numpy as np
import pytest
import torch

from oracle import powersgd_oracle as O
from powersgd_amd import _lib
from powersgd_amd.powersgd import Config, PowerSGD, avg_compressed_size
from powersgd_amd.workloads import CONFIGS, reference_test_model_shapes, resnet50_shapes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    with open(os.path.join(REPO, "include", "psgd.h")) as f:
        header = f.read()
    declared = set(re.findall(r"^\s*(?:int|const char\*)\s+(psgd_\w+)\s*\(", header, re.M))
    assert declared, "no declarations parsed"
    L = _lib.lib()
    for name in sorted(declared):
        assert hasattr(L, name), name
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    assert L.psgd_version() >= 100


SHAPE_SETS = {
    "resnet50": resnet50_shapes(),
    "refmodel": reference_test_model_shapes(),
    "llama": CONFIGS["cfg4_llama_r2_bf16"]["shapes"],
    "mixed": [(16, 8, 3, 3), (16, 8, 3, 3), (3, 200), (64, 16, 1, 1), (16,), (37, 53), (5, 1, 1), (120, 40)],
}


@pytest.mark.parametrize("name", sorted(SHAPE_SETS))
@pytest.mark.parametrize("rank,iters", [(1, 1), (1, 2), (2, 3), (4, 2), (7, 1)])
def test_plan_layout_matches_reference(name, rank, iters):
    shapes = SHAPE_SETS[name]
    plan = _lib.Plan(shapes, rank, iters, _lib.PSGD_F32)
    st = O.codec_init([torch.zeros(s) for s in shapes], rank, iters)
    groups = plan.groups()
    assert [(n, m) for n, m, _, _ in groups] == [tuple(s) for s in st.shapes]
    assert [c for *_, c in groups] == st.counts
    assert [r for _, _, r, _ in groups] == [O.effective_rank(rank, s) for s in st.shapes]
    assert plan.factor_numel() == (st.p_flat.numel(), st.q_flat.numel())
    numels = [int(np.prod(s)) for s in shapes]
    assert plan.output_offsets() == list(np.cumsum([0] + numels[:-1]))
    assert plan.output_numel() == sum(numels)
    rate, unc, comp = plan.compression_rate()
    assert rate == pytest.approx(O.codec_compression_rate(st), rel=1e-12)
    assert plan.workspace_bytes() > 0


@pytest.mark.parametrize("name", sorted(SHAPE_SETS))
@pytest.mark.parametrize("rank,iters,mcr", [(1, 2, 2), (2, 3, 10), (4, 1, 0.5), (4, 2, 2)])
def test_compression_policy_matches_reference(name, rank, iters, mcr):
    cfg = Config(rank, mcr, iters, 0)
    for s in SHAPE_SETS[name]:
        shape = torch.Size(s)
        want = O.compress_decision(shape, rank, iters, mcr)
        assert _lib.should_compress(s, rank, iters, mcr) == want
        assert (shape.numel() / avg_compressed_size(shape, cfg) > mcr) == want


def test_plan_errors_mirror_reference():
    with pytest.raises(IndexError):
        _lib.Plan([], 1, 1, _lib.PSGD_F32)
    with pytest.raises(ValueError):
        _lib.Plan([(4, 4)], 0, 1, _lib.PSGD_F32)
    with pytest.raises(ValueError):
        _lib.Plan([(4, 4)], 1, 17, _lib.PSGD_F32)
    with pytest.raises(RuntimeError):
        _lib.Plan([(4, 4)], 1, 1, 7)
    with pytest.raises(RuntimeError):
        _lib.Plan([(4, 0)], 1, 1, _lib.PSGD_F32)


def test_cpu_tensors_fail_loudly():
    params = [torch.zeros(8, 8)]
    with pytest.raises(RuntimeError, match="GPU"):
        PowerSGD(params, Config(rank=1, min_compression_rate=1, start_compressing_after_num_steps=0))
