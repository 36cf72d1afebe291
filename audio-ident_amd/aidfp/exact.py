"""Exact-identification lane on top of the GPU engine.

Behavioural mirror of audio-ident-service/app/search/exact.py (reference):
clips of at most 5 s are queried as three overlapping sub-windows (:48-52,
:132-173) and merged by consensus (:220-293); longer clips are queried whole
(:176-191, :296-332); candidates below MIN_ALIGNED_HASHES are dropped (:33,
:109), confidence = min(h / 20, 1) (:340-353), results sorted by confidence
(stable) and cut to max_results (:118-121), then enriched with track metadata
(:447-496; missing tracks dropped). tests/test_glue_parity.py replays vectors
captured from the reference (tests/golden/ref_glue.json) through this module.

Differences by design: the query function and the metadata lookup are
injectable (the reference hard-wires olaf_query and Postgres); the default
query function is aidfp.fingerprint.olaf_query (GPU engine) and the default
lookup returns the track UUID itself.
"""

from __future__ import annotations

import logging
import statistics
import uuid
from dataclasses import dataclass
from typing import Any, Awaitable, Callable, Iterable, Sequence

from .fingerprint import OlafError, OlafMatch

logger = logging.getLogger(__name__)

MIN_ALIGNED_HASHES = 8
STRONG_MATCH_HASHES = 20
SHORT_CLIP_THRESHOLD_SEC = 5.0
SUB_WINDOWS = ((0.0, 3.5), (0.75, 4.25), (1.5, 5.0))
SAMPLE_RATE = 16000
BYTES_PER_SAMPLE = 4

QueryFn = Callable[[bytes], Awaitable[list[OlafMatch]]]
LookupFn = Callable[[list[uuid.UUID]], Awaitable[dict[uuid.UUID, Any]]]


@dataclass
class ScoredCandidate:
    track_uuid: uuid.UUID
    aligned_hashes: int
    offset_seconds: float | None
    confidence: float = 0.0


@dataclass
class ExactMatch:
    """Field-for-field the reference's app.schemas.search.ExactMatch (:27-33)."""

    track: Any
    confidence: float
    offset_seconds: float | None
    aligned_hashes: int


def pcm_duration_sec(pcm: bytes, sample_rate: int = SAMPLE_RATE) -> float:
    return (len(pcm) // BYTES_PER_SAMPLE) / sample_rate


def extract_pcm_window(pcm: bytes, start_sec: float, stop_sec: float, sample_rate: int = SAMPLE_RATE) -> bytes:
    """Byte slice [start, stop) at 16 kHz f32le, clamped to the data (reference :374-399)."""
    lo = int(start_sec * sample_rate) * BYTES_PER_SAMPLE
    hi = int(stop_sec * sample_rate) * BYTES_PER_SAMPLE
    lo = min(max(lo, 0), len(pcm))
    hi = max(lo, min(hi, len(pcm)))
    return pcm[lo:hi]


def normalize_confidence(aligned_hashes: int) -> float:
    return 0.0 if aligned_hashes <= 0 else min(aligned_hashes / STRONG_MATCH_HASHES, 1.0)


def _as_uuid(path: str) -> uuid.UUID | None:
    try:
        return uuid.UUID(path)
    except ValueError:
        logger.warning("non-UUID reference_path: %s", path)
        return None


def _group(tagged: Iterable[tuple[int, OlafMatch]]) -> dict[str, list[tuple[int, OlafMatch]]]:
    groups: dict[str, list[tuple[int, OlafMatch]]] = {}
    for tag, m in tagged:
        groups.setdefault(m.reference_path.strip(), []).append((tag, m))
    return groups


def matches_to_candidates(matches: Sequence[OlafMatch]) -> list[ScoredCandidate]:
    """Full-clip aggregation: per track, summed match counts and median reference start."""
    out = []
    for path, rows in _group((0, m) for m in matches).items():
        tid = _as_uuid(path)
        if tid is None:
            continue
        starts = [m.reference_start for _, m in rows]
        out.append(ScoredCandidate(tid, sum(m.match_count for _, m in rows), statistics.median(starts)))
    return out


def consensus_score(window_results: Sequence[Sequence[OlafMatch]]) -> list[ScoredCandidate]:
    """Sub-window consensus: tracks seen in >= 2 windows keep the summed count, single-window
    tracks keep half of it (at least 1); offset = median of the raw reference starts."""
    tagged = ((w, m) for w, ms in enumerate(window_results) for m in ms)
    out = []
    for path, rows in _group(tagged).items():
        tid = _as_uuid(path)
        if tid is None:
            continue
        total = sum(m.match_count for _, m in rows)
        offset = statistics.median([m.reference_start for _, m in rows])
        windows = {w for w, _ in rows}
        out.append(ScoredCandidate(tid, total if len(windows) >= 2 else max(total // 2, 1), offset))
    return out


async def _default_lookup(ids: list[uuid.UUID]) -> dict[uuid.UUID, Any]:
    return {i: i for i in ids}


async def _default_query(pcm: bytes) -> list[OlafMatch]:
    from .fingerprint import olaf_query

    return await olaf_query(pcm)


async def _query_subwindows(pcm: bytes, duration: float, query: QueryFn,
                            sample_rate: int = SAMPLE_RATE) -> list[ScoredCandidate]:
    per_window: list[list[OlafMatch]] = []
    for a, b in SUB_WINDOWS:
        stop = min(b, duration)
        piece = extract_pcm_window(pcm, a, stop, sample_rate) if a < stop else b""
        if not piece:
            per_window.append([])
            continue
        try:
            per_window.append(await query(piece))
        except OlafError:
            logger.exception("sub-window [%.2f, %.2f] query failed", a, stop)
            per_window.append([])
    return consensus_score(per_window)


async def _query_full(pcm: bytes, query: QueryFn) -> list[ScoredCandidate]:
    try:
        return matches_to_candidates(await query(pcm))
    except OlafError:
        logger.exception("full-clip query failed")
        return []


def rank(candidates: list[ScoredCandidate], max_results: int) -> list[ScoredCandidate]:
    kept = [c for c in candidates if c.aligned_hashes >= MIN_ALIGNED_HASHES]
    for c in kept:
        c.confidence = normalize_confidence(c.aligned_hashes)
    kept.sort(key=lambda c: c.confidence, reverse=True)  # stable, like the reference
    return kept[:max_results]


async def enrich(top: list[ScoredCandidate], lookup: LookupFn) -> list[ExactMatch]:
    if not top:
        return []
    found = await lookup([c.track_uuid for c in top])
    out = []
    for c in top:
        meta = found.get(c.track_uuid)
        if meta is None:
            logger.warning("track %s not in metadata store, dropped", c.track_uuid)
            continue
        out.append(ExactMatch(meta, c.confidence, c.offset_seconds, c.aligned_hashes))
    return out


async def run_exact_lane(pcm_16k: bytes, max_results: int = 10, *, query: QueryFn | None = None,
                         lookup: LookupFn | None = None, sample_rate: int = SAMPLE_RATE) -> list[ExactMatch]:
    """Reference semantics of run_exact_lane (exact.py:70-124) over the GPU engine.

    With the default query function the whole lane (fan-out, match, consensus, ranking) is one
    batched engine call (run_exact_lane_batch); an injected `query` runs the per-window path."""
    if not pcm_16k:
        return []
    if query is None:
        return (await run_exact_lane_batch([pcm_16k], max_results, lookup=lookup))[0]
    duration = pcm_duration_sec(pcm_16k, sample_rate)  # sample_rate: the reference's SAMPLE_RATE (16 kHz)
    if duration <= SHORT_CLIP_THRESHOLD_SEC:
        scored = await _query_subwindows(pcm_16k, duration, query, sample_rate)
    else:
        scored = await _query_full(pcm_16k, query)
    return await enrich(rank(scored, max_results), lookup or _default_lookup)


def candidates_from_rows(rows, names: dict[int, str], max_results: int) -> list[ScoredCandidate]:
    """Engine exact-lane rows (rank order) -> ScoredCandidate list: rows of tracks without a name
    (not in the service's map) are dropped before the top-N cut, as the per-window path drops
    them before the consensus (a track is its own group, so the survivors' order is the same)."""
    out = []
    for r in rows:
        name = names.get(int(r["track"]))
        tid = _as_uuid(name) if name is not None else None
        if tid is None:
            continue
        out.append(ScoredCandidate(tid, int(r["aligned_hashes"]), float(r["offset_seconds"]), float(r["confidence"])))
        if len(out) == max_results:
            break
    return out


async def run_exact_lane_batch(clips: Sequence[bytes], max_results: int = 10, *, service=None,
                               lookup: LookupFn | None = None) -> list[list[ExactMatch]]:
    """run_exact_lane for a batch of 16 kHz f32le clips in one engine call (aid_exact_lane):
    sub-window fan-out, K1-K5 and the consensus/threshold/ranking kernel on the GPU; only the
    metadata lookup runs here. An engine failure, including an engine that cannot start
    (OlafError), gives [] for every clip: the reference logs a failed olaf query and carries on
    (exact.py:163-171 sub-windows, :186-190 full clip)."""
    import asyncio

    from .fingerprint import get_service

    if not clips:
        return []
    try:
        svc = service or get_service()
        ranked = await asyncio.get_running_loop().run_in_executor(None, svc.exact_batch, list(clips), max_results)
    except OlafError:
        logger.exception("exact lane: fingerprint engine unavailable")
        ranked = [[] for _ in clips]
    except Exception:
        logger.exception("batched exact lane failed")
        ranked = [[] for _ in clips]
    return [await enrich(r, lookup or _default_lookup) for r in ranked]
