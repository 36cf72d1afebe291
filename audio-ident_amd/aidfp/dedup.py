"""Chromaprint content-duplicate detection on the GPU -- drop-in for
audio-ident-service/app/audio/dedup.py.

The reference (dedup.py:169-222) SELECTs every track within +-10 % of the upload's duration
and scores each stored raw Chromaprint fingerprint against the new one in a Python loop
(`_fingerprint_similarity`, :127-166: bitwise Hamming agreement over the overlapping
words, times min_len/max_len). Here the catalog of fingerprints lives in HBM
(`ContentIndex`, C ABI aid_dedup_*) and one launch scores a whole batch of uploads against
it (K7 `dedup_scan`, csrc/dedup.hip); the score is the same binary64 value and the same
winner (earliest of the best, strict >) as the reference (tests/test_gpu_dedup.py against
vectors captured from the reference, tests/golden/ref_dedup.json).

Kept from the reference unchanged in meaning: `f32le_to_s16le` (:41-53; numpy, host),
`check_file_duplicate` stays a SQL lookup (not on the GPU), and fpcalc itself stays external.
"""

from __future__ import annotations

import ctypes
import threading
import uuid
from typing import Sequence

import numpy as np

from ._lib import check


def f32le_to_s16le(pcm_f32le: bytes) -> bytes:
    """f32le PCM -> s16le PCM (dedup.py:41-53)."""
    samples = np.frombuffer(pcm_f32le, dtype=np.float32)
    return np.clip(samples * 32767, -32768, 32767).astype(np.int16).tobytes()


def parse_fingerprint(fp: str | None) -> np.ndarray | None:
    """Raw Chromaprint 'a,b,c' -> uint32 words (two's complement of signed ints), as the
    reference parses it (`int(x) for x in fp.split(",")`); None when that raises ValueError."""
    if fp is None:
        return None
    try:
        vals = [int(x) for x in fp.split(",")]
    except ValueError:
        return None
    return np.array([v & 0xFFFFFFFF for v in vals], dtype=np.uint32)


def _packed(arrs: Sequence[np.ndarray]):
    off = np.zeros(len(arrs) + 1, dtype=np.int64)
    if arrs:
        off[1:] = np.cumsum([len(a) for a in arrs])
    words = np.concatenate(arrs).astype(np.uint32) if arrs and off[-1] else np.zeros(1, np.uint32)
    return np.ascontiguousarray(words), off


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


class ContentIndex:
    """Device-resident catalog of (track id, raw fingerprint, duration) in insertion order."""

    def __init__(self, engine):
        self.eng = engine
        self.ids: list = []
        check(engine._lib.aid_dedup_reset(engine._h))

    def add(self, ids: Sequence, fingerprints: Sequence[str | None], durations: Sequence[float | None]) -> int:
        """Append tracks; those without a fingerprint or duration are skipped, as the reference's
        SQL filter skips them (dedup.py:196-197). Returns how many were stored."""
        keep_ids, arrs, durs = [], [], []
        for i, fp, d in zip(ids, fingerprints, durations):
            if fp is None or d is None:
                continue
            a = parse_fingerprint(fp)
            keep_ids.append(i)
            arrs.append(a if a is not None else np.zeros(0, np.uint32))  # unparsable: scores 0.0
            durs.append(float(d))
        if not arrs:
            return 0
        words, off = _packed(arrs)
        dur = np.ascontiguousarray(durs, dtype=np.float64)
        check(self.eng._lib.aid_dedup_add(self.eng._h, _p(words), _p(off), _p(dur), len(arrs)))
        self.ids += keep_ids
        return len(arrs)

    def __len__(self) -> int:
        return len(self.ids)

    def scan(self, fingerprints: Sequence[str], durations: Sequence[float]):
        """Best entry per upload within +-10 % duration: (ids or None, scores)."""
        arrs = [parse_fingerprint(f) for f in fingerprints]
        arrs = [a if a is not None else np.zeros(0, np.uint32) for a in arrs]
        words, off = _packed(arrs)
        dur = np.ascontiguousarray([float(d) for d in durations], dtype=np.float64)
        nq = len(arrs)
        idx = np.zeros(max(1, nq), dtype=np.int64)
        sim = np.zeros(max(1, nq), dtype=np.float64)
        check(self.eng._lib.aid_dedup_scan(self.eng._h, _p(words), _p(off), _p(dur), nq, _p(idx), _p(sim)))
        return [self.ids[i] if i >= 0 else None for i in idx[:nq]], sim[:nq]

    def check(self, fingerprint: str, duration: float, threshold: float = 0.85):
        """check_content_duplicate against this catalog: best id if its score >= threshold."""
        ids, sims = self.scan([fingerprint], [duration])
        if ids[0] is not None and sims[0] >= threshold:
            return ids[0]
        return None

    def check_batch(self, fingerprints: Sequence[str], durations: Sequence[float], threshold: float = 0.85):
        ids, sims = self.scan(fingerprints, durations)
        return [i if i is not None and s >= threshold else None for i, s in zip(ids, sims)]


_engine = None
_engine_lock = threading.Lock()


def _default_engine():
    global _engine
    with _engine_lock:
        if _engine is None:
            from .engine import Engine

            _engine = Engine(16000)
        return _engine


def fingerprint_similarity_batch(pairs: Sequence[tuple[str, str]], engine=None) -> np.ndarray:
    """`_fingerprint_similarity` of many pairs in one launch (K7 pairs kernel)."""
    eng = engine or _default_engine()
    a_arr, b_arr, bad = [], [], []
    for k, (x, y) in enumerate(pairs):
        a, b = parse_fingerprint(x), parse_fingerprint(y)
        if a is None or b is None:
            bad.append(k)
            a = b = np.zeros(0, np.uint32)
        a_arr.append(a)
        b_arr.append(b)
    aw, ao = _packed(a_arr)
    bw, bo = _packed(b_arr)
    n = len(a_arr)
    out = np.zeros(max(1, n), dtype=np.float64)
    check(eng._lib.aid_dedup_pairs(eng._h, _p(aw), _p(ao), _p(bw), _p(bo), n, _p(out)))
    out = out[:n]
    out[bad] = 0.0
    return out


def _fingerprint_similarity(fp1: str, fp2: str) -> float:
    """dedup.py:127-166, scored on the GPU."""
    return float(fingerprint_similarity_batch([(fp1, fp2)])[0])


def _candidate_statement(duration: float):
    """The reference's SELECT (dedup.py:190-202); needs the service's Track model."""
    from sqlalchemy import select

    from app.models.track import Track  # noqa: PLC0415 -- available inside audio-ident-service

    return select(Track.id, Track.chromaprint_fingerprint, Track.chromaprint_duration).where(
        Track.chromaprint_fingerprint.isnot(None),
        Track.chromaprint_duration.isnot(None),
        Track.chromaprint_duration >= duration * 0.9,
        Track.chromaprint_duration <= duration * 1.1,
    )


async def check_content_duplicate(session, fingerprint: str, duration: float, threshold: float = 0.85,
                                  engine=None) -> uuid.UUID | None:
    """Drop-in for dedup.py:169-222. `session` is either a `ContentIndex` (catalog resident on
    the GPU: one scan, no SQL) or the service's AsyncSession (the reference's SELECT, then the
    returned rows are scored on the GPU in one launch)."""
    if isinstance(session, ContentIndex):
        return session.check(fingerprint, duration, threshold)
    result = await session.execute(_candidate_statement(duration))
    rows = [r for r in result.all() if r[1] is not None]
    if not rows:
        return None
    sims = fingerprint_similarity_batch([(fingerprint, r[1]) for r in rows], engine)
    best_id, best = None, 0.0
    for (track_id, _fp, _d), s in zip(rows, sims):  # strict >: the earliest of the best wins
        if s > best:
            best, best_id = float(s), track_id
    if best >= threshold and best_id is not None:
        return best_id
    return None
