"""Record every parity comparison's observed error next to its bound.

``check(err, tol, *ctx)`` asserts ``err <= tol`` and appends one JSON line (test id, context,
error, tolerance) to ``$PSGD_PARITY_LOG`` (default ``gpurun_out/parity_errors.jsonl`` in the
repository, created on demand). Works from spawned worker processes too: the test id comes
from ``PYTEST_CURRENT_TEST``, which the workers inherit. ``tools/parity_summary.py`` reduces
the log to the maximum error per test, which is what DESIGN.md quotes against each bound.
"""
from __future__ import annotations

import json
import os

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOG = os.environ.get("PSGD_PARITY_LOG") or os.path.join(_REPO, "gpurun_out", "parity_errors.jsonl")


def record(err: float, tol: float, *ctx) -> None:
    test = os.environ.get("PYTEST_CURRENT_TEST", "?").split(" ")[0]
    try:
        os.makedirs(os.path.dirname(LOG), exist_ok=True)
        with open(LOG, "a") as f:
            f.write(json.dumps({"test": test, "ctx": [str(c) for c in ctx], "err": float(err),
                                "tol": float(tol)}) + "\n")
    except OSError:
        pass


def check(err: float, tol: float, *ctx) -> None:
    record(err, tol, *ctx)
    assert err <= tol, (ctx, err, tol)
