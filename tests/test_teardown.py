"""Ordered teardown at interpreter exit (aidfp.engine._shutdown): services registered with on_shutdown are closed
from one atexit hook that runs BEFORE torch's own (it is registered after torch is imported), every live engine is
destroyed there, and Engine.__del__ does nothing afterwards -- no HIP call from interpreter or C-runtime teardown
(the round-4 exit-time SIGSEGV under rocprofv3). CPU only: fake engines stand in for the library."""

import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

SCRIPT = r"""
import atexit, sys
sys.path.insert(0, {pkg!r})
import torch
from aidfp import engine as E

order = []
atexit.register(lambda: print("late-hook", order, flush=True))  # registered first: runs after ours

class Lib:
    def aid_engine_destroy(self, h):
        order.append("destroy")

class Svc:
    def close(self):
        order.append("service")

eng = E.Engine.__new__(E.Engine)  # no device here: a handle and a fake library
eng._h, eng._lib = 1, Lib()
E._live.add(eng)
svc = Svc()
E.on_shutdown(svc)
print("registered", flush=True)
"""


def test_shutdown_order_and_no_late_calls():
    out = subprocess.run([sys.executable, "-c", SCRIPT.format(pkg=str(ROOT / "audio-ident_amd"))],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.split()
    assert "registered" in lines
    # the service closes first, then the engine is destroyed exactly once, all before the earlier hooks run
    assert "late-hook ['service', 'destroy']" in out.stdout, out.stdout


def test_del_is_a_noop_after_shutdown():
    from aidfp import engine as E

    calls = []

    class Lib:
        def aid_engine_destroy(self, h):
            calls.append(h)

    eng = E.Engine.__new__(E.Engine)
    eng._h, eng._lib = 7, Lib()
    saved = E._shutdown_done
    try:
        E._shutdown_done = True
        eng.__del__()
        assert calls == []
    finally:
        E._shutdown_done = saved
    eng.close()
    assert calls == [7]


def test_host_concat_threaded_equals_concatenate(monkeypatch):
    """The multi-threaded host batch copy (large coalesced batches) lays the clips out exactly as np.concatenate."""
    import numpy as np

    from aidfp import engine as E

    rng = np.random.default_rng(3)
    arrs = [rng.random(int(rng.integers(0, 50000))).astype(np.float32) for _ in range(37)]
    out = np.empty(sum(len(a) for a in arrs), np.float32)
    monkeypatch.setattr(E, "_COPY_MIN", 1)
    E._concat_into(arrs, out)
    assert np.array_equal(out, np.concatenate(arrs))
    small = np.empty(10, np.float32)
    E._concat_into([np.arange(4, dtype=np.float32), np.arange(6, dtype=np.float32)], small)
    assert np.array_equal(small, np.concatenate([np.arange(4), np.arange(6)]).astype(np.float32))
