"""The output buffer cache (csrc/psgd_host.cpp OutputSlab) on CPU tensors: the previous call's
buffer may be handed out again only when NO reference to any of its views survives. The
reference returns fresh tensors every call (powersgd.py:153), so every way a caller can keep
an output — a Python variable, ``p.grad``, autograd's saved tensors, a derived view,
``.detach()``, the storage object — must force a fresh buffer."""
import torch

from powersgd_amd import _psgd_host as H

SHAPES = [[64, 3, 7, 7], [64], [256, 64, 1, 1], [1000, 2048], [1000]]


def _slab():
    s = H.OutputSlab(SHAPES, 0, -1)  # device -1: CPU (the policy is device-independent)
    s.get()
    return s


def test_layout_views_of_one_flat_buffer():
    s = H.OutputSlab(SHAPES, 0, -1)
    outs = s.get()
    off = 0
    for o, shp in zip(outs, SHAPES):
        assert list(o.shape) == shp and o.is_contiguous()
        assert o.data_ptr() == s.flat.data_ptr() + off * 4
        off += o.numel()


def test_reuse_when_nothing_holds_the_outputs():
    s = _slab()
    for _ in range(5):
        s.get()
    assert s.fresh == 1


def test_python_reference_forces_fresh_buffer():
    s = _slab()
    outs = s.get()
    keep = outs[2]
    del outs
    new = s.get()
    assert s.fresh == 2 and new[2].data_ptr() != keep.data_ptr()


def test_p_grad_reference_forces_fresh_buffer():
    s = _slab()
    p = torch.nn.Parameter(torch.zeros(SHAPES[3]))
    p.grad = s.get()[3]
    s.get()
    assert s.fresh == 2
    p.grad = None
    s.get()
    s.get()
    assert s.fresh == 2  # the second buffer was never held: reused from then on


def test_autograd_saved_tensor_forces_fresh_buffer():
    s = _slab()
    w = torch.ones(SHAPES[0], requires_grad=True)
    loss = (s.get()[0] * w).sum()  # saves the output for backward
    s.get()
    assert s.fresh == 2
    del loss


def test_derived_view_and_detach_force_fresh_buffer():
    s = _slab()
    a = s.get()[4][:10]
    s.get()
    assert s.fresh == 2
    del a
    b = s.get()[1].detach()
    s.get()
    assert s.fresh == 3
    del b
    st = s.get()[1].untyped_storage()
    s.get()
    assert s.fresh == 4
    del st


def test_list_of_outputs_held_forces_fresh_buffer():
    s = _slab()
    held = s.get()
    again = s.get()
    assert s.fresh == 2 and held[0].data_ptr() != again[0].data_ptr()
