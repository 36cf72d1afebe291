"""GPU Chromaprint dedup (K7, aid_dedup_*) vs the reference's own outputs
(tests/golden/ref_dedup.json: dedup.py `_fingerprint_similarity` values and
`check_content_duplicate` decisions, captured by tests/golden/make_dedup_fixtures.py)."""

import asyncio
import json
import uuid
from pathlib import Path

import numpy as np
import pytest

from aidfp import dedup

pytestmark = pytest.mark.gpu
GOLD = json.loads((Path(__file__).resolve().parent / "golden" / "ref_dedup.json").read_text())


def test_similarity_equals_reference(gpu_engine):
    pairs = [(s["fp1"], s["fp2"]) for s in GOLD["similarity"]]
    got = dedup.fingerprint_similarity_batch(pairs, gpu_engine)
    want = np.array([s["sim"] for s in GOLD["similarity"]], dtype=np.float64)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), np.nonzero(got != want)


def _index(eng):
    idx = dedup.ContentIndex(eng)
    cat = GOLD["catalog"]
    idx.add([c["id"] for c in cat], [c["fp"] for c in cat], [c["duration"] for c in cat])
    return idx


def test_scan_decisions_equal_reference(gpu_engine):
    idx = _index(gpu_engine)
    assert len(idx) == len(GOLD["catalog"]) - 2  # the entries without fingerprint / duration
    for q in GOLD["queries"]:
        assert idx.check(q["fingerprint"], q["duration"], q["threshold"]) == q["result"], q["duration"]
    # one launch for the whole batch, per-query thresholds applied on the host
    ids, sims = idx.scan([q["fingerprint"] for q in GOLD["queries"]], [q["duration"] for q in GOLD["queries"]])
    for q, i, s in zip(GOLD["queries"], ids, sims):
        assert (i if i is not None and s >= q["threshold"] else None) == q["result"]


class _Result:
    def __init__(self, rows):
        self.rows = rows

    def all(self):
        return self.rows


class _Session:
    """Stands in for the service's AsyncSession: applies the SELECT's duration bounds."""

    def __init__(self, catalog, duration):
        self.catalog, self.duration = catalog, duration

    async def execute(self, _stmt):
        lo, hi = self.duration * 0.9, self.duration * 1.1
        return _Result([(c["id"], c["fp"], c["duration"]) for c in self.catalog
                        if c["fp"] is not None and c["duration"] is not None and lo <= c["duration"] <= hi])


def test_session_path_equals_reference(gpu_engine, monkeypatch):
    monkeypatch.setattr(dedup, "_candidate_statement", lambda d: None)
    for q in GOLD["queries"]:
        got = asyncio.run(dedup.check_content_duplicate(_Session(GOLD["catalog"], q["duration"]), q["fingerprint"],
                                                        q["duration"], q["threshold"], engine=gpu_engine))
        assert got == q["result"]


def test_large_catalog_batch_consistency(gpu_engine):
    """Many chunks: batch results equal one-at-a-time results, and planted near-duplicates win."""
    rng = np.random.default_rng(7)
    n = 3000
    fps = [rng.integers(0, 2**32, size=int(rng.integers(100, 600)), dtype=np.uint64) for _ in range(n)]
    durs = rng.uniform(30, 300, size=n).round(3)
    idx = dedup.ContentIndex(gpu_engine)
    to_s = lambda a: ",".join(str(int(v) - (1 << 32) if v >= (1 << 31) else int(v)) for v in a)
    idx.add([str(uuid.UUID(int=i + 1)) for i in range(n)], [to_s(f) for f in fps], durs.tolist())
    src = rng.integers(0, n, size=64)
    qs, qd = [], []
    for s in src:
        q = fps[s].copy()
        q[::7] ^= 1 << 5
        qs.append(to_s(q))
        qd.append(float(durs[s]) * 1.03)
    ids, sims = idx.scan(qs, qd)
    for k, s in enumerate(src):
        assert ids[k] == str(uuid.UUID(int=int(s) + 1))
        assert sims[k] > 0.99
        one_id, one_sim = idx.scan([qs[k]], [qd[k]])
        assert one_id[0] == ids[k] and one_sim[0] == sims[k]
