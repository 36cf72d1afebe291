"""bench.py's host-side helpers on CPU: the parity check it prints next to the headline (the batch's
hashes against the C oracle) and the cpu_baseline leg. The GPU engine is replaced by a stub that
serves records; the GPU run itself is `python bench.py` (GPU box)."""

import numpy as np

import bench
import oracle as O
from aidfp import synth


class _Records:
    """Stands in for aidfp.engine.Engine: hashes(c) -> the uint64 records of clip c."""

    def __init__(self, recs):
        self.recs = recs

    def hashes(self, c):
        return self.recs[c]


def _clips(n=3, seconds=2.0):
    return np.stack([synth.synth(t, 0, int(seconds * bench.SR), bench.SR, snr_db=20.0) for t in range(n)])


def test_parity_bit_exact_and_mismatch():
    x = _clips()
    ref = O.fingerprint_batch(x, 512)
    assert all(len(r) > 0 for r in ref)
    p = bench.parity(_Records([r.copy() for r in ref]), x, ref)
    assert p["bit_exact"] and p["clips"] == 3 and p["hashes"] == sum(len(r) for r in ref)
    bad = [r.copy() for r in ref]
    bad[1][len(bad[1]) // 2] ^= np.uint64(1)  # one hash bit of one record
    p = bench.parity(_Records(bad), x, ref)
    assert not p["bit_exact"] and p["mismatched_clips"] == [1]
    short = [r.copy() for r in ref]
    short[2] = short[2][:-1]  # a missing record
    assert bench.parity(_Records(short), x, ref)["mismatched_clips"] == [2]


def test_parity_runs_the_oracle_when_no_reference_is_given():
    x = _clips(n=2)
    ref = O.fingerprint_batch(x, 512)
    p = bench.parity(_Records(ref), x)
    assert p["bit_exact"] and p["clips"] == 2


def test_cpu_baseline_returns_the_batch_records():
    x = _clips(n=2, seconds=1.0)
    ref, cpu = bench.cpu_baseline(x, min_s=0.0)
    want = O.fingerprint_batch(x, 512)
    assert len(ref) == 2 and all(np.array_equal(a, b) for a, b in zip(ref, want))
    assert cpu["unit"] == "audio-s/s" and cpu["kind"] == "port" and cpu["value"] > 0 and cpu["cores"] >= 1
    assert "pass(es)" in cpu["sample"]


def test_cpu_baseline_names_the_host_and_numpy_leg():
    x = _clips(n=2, seconds=1.0)
    _, cpu = bench.cpu_baseline(x, min_s=0.0)
    assert cpu["cpu_model"] and cpu["cpus_visible"] >= cpu["cores"] >= 1
    assert cpu["numpy_scipy"]["value_1proc"] > 0 and cpu["numpy_scipy"]["value_pool"] > 0


def test_launch_plan():
    assert bench.launch_plan(1, {}) == "run"
    assert bench.launch_plan(2, {}) == "spawn"
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == "run"
    assert bench.launch_plan(2, {"WORLD_SIZE": "1"}) == "error"


def _bench(args, env_extra=None):
    import json
    import os
    import subprocess
    import sys

    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, str(bench.ROOT / "bench.py"), *args], env=env, capture_output=True,
                       text=True, timeout=240)
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, lines, r.stderr


def test_gpus_2_spawns_two_ranks():
    """`python bench.py --gpus 2` (the driver's N=1-style invocation with N=2) starts 2 ranks itself."""
    rc, lines, err = _bench(["--gpus", "2", "--dry-run"])
    assert rc == 0, err[-2000:]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)


def test_world_size_mismatch_fails():
    rc, lines, err = _bench(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines and "WORLD_SIZE=3" in err
