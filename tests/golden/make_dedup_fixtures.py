"""Capture the reference's Chromaprint content-dedup behaviour as JSON vectors.

Runs ONLY in the build container: it imports the reference Python from /root/reference
(read-only; nothing of it is copied or shipped) with the same import shims as
make_glue_fixtures.py. Output: tests/golden/ref_dedup.json -- inputs and outputs of
  app/audio/dedup.py  _fingerprint_similarity   (:127-166)
                      check_content_duplicate   (:169-222), run against a fake AsyncSession
                      that applies the statement's own compiled duration bounds
                      (duration * 0.9 <= d <= duration * 1.1, :193-201) and returns the
                      surviving rows in catalog order.
                      f32le_to_s16le            (:41-53)

Run: python tests/golden/make_dedup_fixtures.py
"""

from __future__ import annotations

import asyncio
import base64
import json
import sys
import uuid
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent))
from make_glue_fixtures import _shims  # noqa: E402

OUT = Path(__file__).resolve().parent / "ref_dedup.json"


def fp_str(a) -> str:
    return ",".join(str(int(x)) for x in a)


class _Result:
    def __init__(self, rows):
        self._rows = rows

    def all(self):
        return list(self._rows)


class FakeSession:
    """Executes the reference's SELECT over an in-memory catalog: the WHERE clause's
    bound parameters (the two duration bounds) are taken from the compiled statement."""

    def __init__(self, catalog):
        self.catalog = catalog  # [(uuid, fp or None, dur or None)]
        self.bounds = None

    async def execute(self, stmt):
        params = stmt.compile().params
        lo = min(v for v in params.values() if isinstance(v, float))
        hi = max(v for v in params.values() if isinstance(v, float))
        self.bounds = (lo, hi)
        rows = [(i, f, d) for i, f, d in self.catalog if f is not None and d is not None and lo <= d <= hi]
        return _Result(rows)


def main() -> None:
    _shims()
    from app.audio import dedup as dd

    rng = np.random.default_rng(20260101)
    out: dict = {"source": "MacPhobos/audio-ident reference, captured by tests/golden/make_dedup_fixtures.py"}

    # ---- pairwise similarity
    sims = []
    def add(a, b):
        sims.append({"fp1": a, "fp2": b, "sim": dd._fingerprint_similarity(a, b)})
    for la, lb in [(1, 1), (5, 5), (100, 100), (100, 97), (1400, 1500), (3, 900), (64, 65), (777, 777)]:
        a = rng.integers(-2**31, 2**31, size=la)
        b = rng.integers(-2**31, 2**31, size=lb)
        add(fp_str(a), fp_str(b))
        c = a.copy()[: lb]
        flips = rng.integers(0, 32, size=len(c))
        c = ((c.astype(np.int64) ^ (1 << flips)) + 2**31) % 2**32 - 2**31  # one bit flipped per word
        add(fp_str(a), fp_str(c))
        add(fp_str(a), fp_str(a))
    for a, b in [("", "1,2"), ("1,2", ""), ("1,x,3", "1,2,3"), ("7", "7"), ("-1", "4294967295"), ("0,0", "-1,-1")]:
        add(a, b)
    out["similarity"] = sims

    # ---- catalog scan (check_content_duplicate)
    n_cat = 60
    base = [rng.integers(-2**31, 2**31, size=int(rng.integers(200, 1500))) for _ in range(n_cat)]
    durs = [float(np.round(rng.uniform(30.0, 300.0), 3)) for _ in range(n_cat)]
    ids = [str(uuid.UUID(int=int(rng.integers(1, 2**62)) * 7919)) for _ in range(n_cat)]
    catalog = [(ids[i], fp_str(base[i]), durs[i]) for i in range(n_cat)]
    catalog[3] = (ids[3], None, durs[3])          # no fingerprint stored
    catalog[4] = (ids[4], fp_str(base[4]), None)  # no duration stored
    catalog[10] = (ids[10], fp_str(base[9]), durs[9])  # exact duplicate of 9, later in order
    cases = []
    for qi in range(40):
        src = int(rng.integers(0, n_cat))
        q = base[src].copy()
        kind = qi % 4
        if kind == 1:  # near-duplicate: ~5 % of bits flipped, slightly different length
            mask = rng.random((len(q), 32)) < 0.05
            flips = (mask * (1 << np.arange(32))).sum(axis=1)
            q = ((q.astype(np.int64) ^ flips) + 2**31) % 2**32 - 2**31
            q = q[: max(1, len(q) - int(rng.integers(0, 20)))]
        elif kind == 2:  # unrelated audio
            q = rng.integers(-2**31, 2**31, size=len(q))
        dur = durs[src] * float(rng.choice([1.0, 1.05, 0.95, 1.2, 0.8, 1.1, 0.9]))
        thr = float(rng.choice([0.85, 0.85, 0.6, 0.95, 0.5]))
        sess = FakeSession(catalog)
        got = asyncio.run(dd.check_content_duplicate(sess, fp_str(q), dur, threshold=thr))
        cases.append({"fingerprint": fp_str(q), "duration": dur, "threshold": thr,
                      "bounds": list(sess.bounds), "result": got if got is None else str(got)})
    out["catalog"] = [{"id": i, "fp": f, "duration": d} for i, f, d in catalog]
    out["queries"] = cases

    # ---- f32le -> s16le
    x = np.concatenate([rng.uniform(-1.2, 1.2, size=64), [0.0, -0.0, 1.0, -1.0, 0.99999, -1.00001, 0.5, 1e-9]])
    x = x.astype(np.float32)
    out["s16"] = {"f32le_b64": base64.b64encode(x.tobytes()).decode(),
                  "s16le_b64": base64.b64encode(dd.f32le_to_s16le(x.tobytes())).decode()}
    OUT.write_text(json.dumps(out))
    print(f"wrote {OUT} ({OUT.stat().st_size} bytes): {len(sims)} similarity pairs, {len(cases)} scans")


if __name__ == "__main__":
    main()
