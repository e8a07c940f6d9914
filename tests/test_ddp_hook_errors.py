"""CPU tests of the DDP hook's failure paths (powersgd_amd/ddp.py): an iteration that cannot
aggregate must fail every bucket future it handed to DDP (so DDP's wait raises instead of
hanging) and leave the state clean for the next iteration. The codec itself is replaced by a
stub here (the real one needs a GPU); tests/test_gpu_training.py runs the hook end to end."""
import pytest
import torch

from powersgd_amd.ddp import PowerSGDState, powersgd_hook


class _Bucket:
    """The GradBucket surface the hook uses."""

    def __init__(self, params, last, index=None):
        self._index = int(last) if index is None else index
        self._params = params
        self._grads = [torch.ones_like(p) for p in params]
        self._buf = torch.cat([g.view(-1) for g in self._grads])
        off = 0
        views = []
        for g in self._grads:
            views.append(self._buf[off:off + g.numel()].view(g.shape))
            off += g.numel()
        self._grads = views
        self._last = last

    def parameters(self):
        return self._params

    def gradients(self):
        return self._grads

    def buffer(self):
        return self._buf

    def is_last(self):
        return self._last

    def index(self):
        return self._index


class _Codec:
    def __init__(self, fail=False):
        self.fail = fail

    def aggregate(self, views):
        if self.fail:
            raise RuntimeError("collective failed")
        return [v.clone() for v in views]


class _CpuRuns:
    """The run table the hook builds per bucket layout (bucket offset, parameter, length), with
    the two native passes (psgd_runs_add / psgd_runs_gather) emulated on CPU tensors."""

    def __init__(self, key, buf, grads, idx):
        self.key = key
        self.offs = [(g.data_ptr() - buf.data_ptr()) // buf.element_size() for g in grads]
        self.idx = list(idx)
        self.lens = [g.numel() for g in grads]


def _state(params, codec):
    st = object.__new__(PowerSGDState)  # the constructor builds a GPU codec: bypass it
    st.params = params
    st._index = {id(p): i for i, p in enumerate(params)}
    st.residual = torch.zeros(sum(p.numel() for p in params))
    st.views, off = [], 0
    for p in params:
        st.views.append(st.residual[off:off + p.numel()].view(p.shape))
        off += p.numel()
    st._runs = {}
    st.powersgd = codec
    st._seen = [False] * len(params)
    st._nseen = 0
    st._pending = []
    st._new_runs = lambda key, buf, grads, idx: _CpuRuns(key, buf, grads, idx)

    def ef_add(buf, runs):
        for o, i, n in zip(runs.offs, runs.idx, runs.lens):
            st.views[i].view(-1).add_(buf[o:o + n])

    def gather(pending, outs):
        for buf, runs, _ in pending:
            for o, i, n in zip(runs.offs, runs.idx, runs.lens):
                buf[o:o + n].copy_(outs[i].reshape(-1))

    st._ef_add, st._gather = ef_add, gather
    return st


def _params(n=3):
    return [torch.nn.Parameter(torch.zeros(4, 2)) for _ in range(n)]


def test_complete_iteration_sets_every_future():
    ps = _params()
    st = _state(ps, _Codec())
    f1 = powersgd_hook(st, _Bucket(ps[:2], False))
    assert not f1.done()
    f2 = powersgd_hook(st, _Bucket(ps[2:], True))
    assert f1.done() and f2.done()
    assert torch.equal(f1.value(), torch.ones(16)) and torch.equal(f2.value(), torch.ones(8))
    assert st._nseen == 0 and st._pending == []


def test_failed_aggregate_fails_pending_futures_and_resets():
    ps = _params()
    st = _state(ps, _Codec(fail=True))
    f1 = powersgd_hook(st, _Bucket(ps[:2], False))
    with pytest.raises(RuntimeError, match="collective failed"):
        powersgd_hook(st, _Bucket(ps[2:], True))
    assert f1.done()
    with pytest.raises(RuntimeError, match="collective failed"):
        f1.wait()
    assert st._nseen == 0 and st._pending == [] and not any(st._seen)
    st.powersgd = _Codec()  # the next iteration starts clean
    powersgd_hook(st, _Bucket(ps[:2], False))
    f = powersgd_hook(st, _Bucket(ps[2:], True))
    assert f.done()


def test_parameter_ddp_never_buckets_raises_instead_of_hanging():
    ps = _params()
    st = _state(ps, _Codec())
    f1 = powersgd_hook(st, _Bucket(ps[:1], False))
    with pytest.raises(RuntimeError, match="never reached a DDP bucket"):
        powersgd_hook(st, _Bucket(ps[1:2], True))  # ps[2] never arrives
    with pytest.raises(RuntimeError):
        f1.wait()
    assert st._nseen == 0 and st._pending == []


def test_unknown_parameter_and_double_arrival():
    ps = _params()
    st = _state(ps, _Codec())
    with pytest.raises(RuntimeError, match="was not given"):
        powersgd_hook(st, _Bucket([torch.nn.Parameter(torch.zeros(2))], False))
    f1 = powersgd_hook(st, _Bucket(ps[:1], False))
    with pytest.raises(RuntimeError, match="twice"):
        powersgd_hook(st, _Bucket(ps[:1], False))
    with pytest.raises(RuntimeError):
        f1.wait()
    assert st._nseen == 0


def test_run_tables_one_run_per_parameter_and_only_the_latest_layout_is_kept():
    """A DDP bucket rebuild (new layout under the same bucket index) replaces that bucket's run
    table; a table holds one (bucket offset, parameter, length) run per parameter, nothing per
    element (no index maps: the hook scales past 2^31 gradient elements)."""
    ps = _params()
    st = _state(ps, _Codec())
    powersgd_hook(st, _Bucket(ps[:2], False, index=0))
    powersgd_hook(st, _Bucket(ps[2:], True, index=1))
    assert sorted(st._runs) == [0, 1]
    assert st._runs[0].offs == [0, 8] and st._runs[0].idx == [0, 1] and st._runs[0].lens == [8, 8]
    # rebuilt buckets: parameter 2 moves into bucket 0
    f0 = powersgd_hook(st, _Bucket([ps[2], ps[0]], False, index=0))
    f1 = powersgd_hook(st, _Bucket(ps[1:2], True, index=1))
    assert sorted(st._runs) == [0, 1]
    assert st._runs[0].idx == [2, 0] and st._runs[0].offs == [0, 8] and st._runs[1].idx == [1]
    # the stub codec leaves the residual in place: two iterations of ones accumulated
    assert torch.equal(f0.value(), torch.full((16,), 2.)) and torch.equal(f1.value(), torch.full((8,), 2.))


def test_bucket_dtype_must_match_the_state():
    """A bucket whose dtype differs from the state's gradient dtype would be read and written at
    the wrong element size by the native run kernels: it must raise (and fail the pending
    futures), not launch."""
    ps = _params()
    st = _state(ps, _Codec())
    f1 = powersgd_hook(st, _Bucket(ps[:2], False))
    b = _Bucket(ps[2:], True)
    b._buf = b._buf.to(torch.bfloat16)
    with pytest.raises(RuntimeError, match="bucket dtype"):
        powersgd_hook(st, b)
    with pytest.raises(RuntimeError):
        f1.wait()
    assert st._nseen == 0 and st._pending == []


def test_mixed_parameter_dtypes_are_refused():
    from powersgd_amd import Config
    ps = [torch.nn.Parameter(torch.zeros(4, 2)), torch.nn.Parameter(torch.zeros(4, 2, dtype=torch.bfloat16))]
    with pytest.raises(RuntimeError, match="one gradient dtype"):
        PowerSGDState(Config(rank=1), ps)
