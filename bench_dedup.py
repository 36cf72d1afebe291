#!/usr/bin/env python3
"""bench_dedup.py -- K7 `dedup_scan` (Chromaprint content dedup) on one MI355X.

Workload: a catalog of 100k tracks with raw Chromaprint-shaped fingerprints (7.8 u32 words per
second of audio, fpcalc's rate; durations uniform 30-300 s; 0.5 GB of words resident in HBM)
and a batch of 256 uploads (half near-duplicates of catalog tracks with 3 % of bits flipped and
up to 5 % duration change, half unrelated). One step = one aid_dedup_scan of the batch: every
catalog track within +-10 % duration of an upload is scored (dedup.py:169-222).
Reported: uploads checked/s, pair scores/s, and the compare bandwidth = 8 B per overlapping word
pair scored (query word + catalog word) / kernel time (L2 serves the query words and the catalog
chunks shared by concurrent queries, so this can exceed HBM). cpu_baseline: oracle/fp_dedup.c
(the same scan in C, 1 thread) on 8 uploads.
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=100000)
    ap.add_argument("--uploads", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import ctypes

    from aidfp._lib import check
    from aidfp.engine import Engine

    rng = np.random.default_rng(42)
    durs = rng.uniform(30.0, 300.0, size=args.tracks).round(3)
    lens = np.maximum(1, (durs * 7.8).astype(np.int64))
    off = np.zeros(args.tracks + 1, np.int64)
    off[1:] = np.cumsum(lens)
    words = rng.integers(0, 2**32, size=int(off[-1]), dtype=np.uint32)

    eng = Engine(16000)
    P = lambda a: ctypes.c_void_p(a.ctypes.data)
    check(eng._lib.aid_dedup_reset(eng._h))
    step = 10000
    for a in range(0, args.tracks, step):
        b = min(args.tracks, a + step)
        o = np.ascontiguousarray(off[a:b + 1] - off[a])
        w = np.ascontiguousarray(words[off[a]:off[b]])
        d = np.ascontiguousarray(durs[a:b])
        check(eng._lib.aid_dedup_add(eng._h, P(w), P(o), P(d), b - a))

    src = rng.integers(0, args.tracks, size=args.uploads)
    qs, qd = [], []
    for k, s in enumerate(src):
        if k % 2 == 0:
            q = words[off[s]:off[s + 1]].copy()
            flip = rng.random((len(q), 32)) < 0.03
            q ^= (flip * (1 << np.arange(32, dtype=np.uint64))).sum(axis=1).astype(np.uint32)
            q = q[: max(1, len(q) - int(rng.integers(0, len(q) // 20 + 1)))]
            qs.append(q)
            qd.append(float(durs[s]) * float(rng.uniform(0.95, 1.05)))
        else:
            n = int(rng.uniform(30, 300) * 7.8)
            qs.append(rng.integers(0, 2**32, size=n, dtype=np.uint32))
            qd.append(n / 7.8)
    qoff = np.zeros(len(qs) + 1, np.int64)
    qoff[1:] = np.cumsum([len(q) for q in qs])
    qw = np.ascontiguousarray(np.concatenate(qs))
    qdur = np.ascontiguousarray(qd, dtype=np.float64)
    bi = np.zeros(len(qs), np.int64)
    bs = np.zeros(len(qs), np.float64)

    def scan():
        check(eng._lib.aid_dedup_scan(eng._h, P(qw), P(qoff), P(qdur), len(qs), P(bi), P(bs)))

    for _ in range(args.warmup):
        scan()
    eng.profile_enable(True)
    eng.profile_read(reset=True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        scan()
    wall = time.perf_counter() - t0
    ms, cnt = eng.profile_read(reset=True)["dedup"]
    eng.profile_enable(False)
    k_ms = ms / cnt

    # work actually done: candidate pairs and overlapping words
    pairs, words_cmp = 0, 0
    for q, d in zip(qs, qd):
        m = (durs >= d * 0.9) & (durs <= d * 1.1)
        pairs += int(m.sum())
        words_cmp += int(np.minimum(lens[m], len(q)).sum())
    hits = int(np.sum([bi[k] == src[k] and bs[k] >= 0.85 for k in range(0, len(qs), 2)]))
    false_hits = int(np.sum([bs[k] >= 0.85 for k in range(1, len(qs), 2)]))

    cpu = None
    if not args.no_cpu:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle as O  # CPU baseline only

        cat = [words[off[i]:off[i + 1]] for i in range(args.tracks)]
        t = time.perf_counter()
        cb, cs = O.dedup_scan(cat, durs, qs[:8], qd[:8])
        dt = time.perf_counter() - t
        assert np.array_equal(cb, bi[:8]) and np.array_equal(cs, bs[:8]), "GPU != oracle"
        cpu = {"value": round(8 / dt, 2), "unit": "uploads/s", "cores": 1, "kind": "port",
               "sample": "8 uploads of the batch through oracle/fp_dedup.c (-O2, 1 thread), results equal to the GPU's"}
    print(json.dumps({
        "metric": "Chromaprint content-dedup uploads checked/s vs a 100k-track catalog, 1 GPU",
        "value": round(args.steps * len(qs) / wall, 1), "unit": "uploads/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True,
        "dtype": "u32 popcount, f64 score", "data": "synthetic (random Chromaprint-shaped fingerprints)",
        "config": {"workload": f"{args.tracks} catalog tracks (30-300 s, 7.8 words/s), {len(qs)} uploads per scan",
                   "catalog_words": int(off[-1])},
        "kernel_ms": round(k_ms, 4), "pairs_per_step": pairs, "pair_scores_per_s": round(pairs / (k_ms * 1e-3), 1),
        "compare_bandwidth_GBps": round(8 * words_cmp / (k_ms * 1e-3) / 1e9, 1),
        "near_dup_found": f"{hits}/{len(qs) // 2}", "unrelated_flagged": f"{false_hits}/{len(qs) // 2}",
        "cpu_baseline": cpu,
    }), flush=True)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
