"""GPU-box diagnostic (not part of tests/): repeat the 4-step MT_UBPL run in
eager / graph / serial-stream modes in one process (after the other GPU test
files when run with them) and report which mode's results vary."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tools")]

import pytest  # noqa: E402

pytestmark = pytest.mark.gpu


def test_flake(monkeypatch):
    import determinism as DT
    from ubpl_amd import train as T
    res = {}
    for mode in ("eager", "graph", "serial", "eager_nosplit"):
        for r in range(int(os.environ.get("FLAKE_REPS", "4"))):
            monkeypatch.setenv("UBPL_MODEL_STREAMS", "0" if mode == "serial" else "1")
            out = DT.run(mode == "graph", mode != "eager_nosplit", 4)
            res.setdefault(mode, []).append(out["params"])
    base = res["serial"][0]
    mx = lambda u, v: max(float((a - b).abs().max()) for a, b in zip(u, v))  # noqa: E731
    for mode, runs in res.items():
        print("FLAKE %-14s vs serial[0]: %s" % (mode, ["%.2g" % mx(p, base) for p in runs]), flush=True)
