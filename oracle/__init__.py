"""TEST INFRASTRUCTURE ONLY — CPU oracle for the PowerSGD codec.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product (``powersgd_amd``) never imports it and has no CPU fallback.

``powersgd_oracle`` restates the reference algorithm (epfml/powersgd,
``powersgd/powersgd.py``, ``powersgd/orthogonalization.py``, ``powersgd/utils.py``)
op for op in PyTorch-CPU so that its outputs are bit-identical to the reference
on the same inputs. Parity is pinned by the golden fixtures in ``tests/golden``,
which were produced by running the reference itself (``tests/golden/make_golden.py``).
"""
