"""Drop-in replacement for audio-ident-service/app/audio/fingerprint.py.

Same public surface and error contract as the reference module, but the work
runs in-process on the GPU engine (libaidfp.so) instead of spawning the external
`olaf_c` binary per call:

  reference (fingerprint.py)                  here
  ------------------------------------------  ---------------------------------------
  OlafError, OlafMatch (:26-50)               same names and fields
  olaf_index_track(pcm, uuid) -> bool (:87)   extract on GPU + add postings + persist
  olaf_query(pcm) -> list[OlafMatch] (:158)   extract + K5 match on GPU, count desc
  olaf_delete_track(uuid) -> bool (:222)      tombstone + persist
  _parse_olaf_output/_line/_parts (:273-350)  same parsing (used by the CLI shim)
  OLAF_DB dir (:71-84)                        same dir: index.aidfp + tracks.json

Error contract (reference :102-155, :173-219, :234-270):
  * empty PCM -> False / [] without touching the engine;
  * engine cannot load (no libaidfp.so / no gfx950 GPU) -> OlafError whose message
    says the fingerprint engine binary was not found;
  * a recoverable engine error (bad input, unknown track on delete) -> False / []
    (logged), like a non-zero olaf_c exit code;
  * anything unexpected -> OlafError.
Index writes are serialised by one lock (the reference's LMDB single-writer
rule, :7-8); engine calls run in a worker thread (ctypes releases the GIL), so
the event loop is never blocked.
"""

from __future__ import annotations

import asyncio
import json
import logging
import os
import threading
import uuid
from dataclasses import dataclass
from pathlib import Path

import numpy as np

logger = logging.getLogger(__name__)

SAMPLE_RATE = 16000  # the reference boundary carries 16 kHz mono f32le (fingerprint.py:10)
DEFAULT_DB = "./data/olaf_db"  # reference settings.olaf_lmdb_path default (settings.py:39)


class OlafError(Exception):
    """Raised when the fingerprint engine is unavailable or fails unexpectedly."""


@dataclass
class OlafMatch:
    match_count: int
    query_start: float
    query_stop: float
    reference_path: str
    reference_id: int
    reference_start: float
    reference_stop: float


# ---------------------------------------------------------------- CSV (CLI shim path)

def _parts_to_match(parts: list[str]) -> OlafMatch | None:
    try:
        count, qs, qe, path, rid, rs, re_ = parts[:7]
        return OlafMatch(int(count), float(qs), float(qe), path, int(rid), float(rs), float(re_))
    except (ValueError, IndexError):
        return None


def _parse_olaf_line(line: str) -> OlafMatch | None:
    for sep in (",", ";"):
        parts = [p.strip() for p in line.split(sep)]
        if len(parts) >= 7:
            return _parts_to_match(parts)
    return None


def _parse_olaf_output(stdout: str) -> list[OlafMatch]:
    rows = [_parse_olaf_line(ln.strip()) for ln in stdout.strip().splitlines() if ln.strip()]
    out = [r for r in rows if r is not None]
    out.sort(key=lambda m: m.match_count, reverse=True)
    return out


def format_match(m: OlafMatch) -> str:
    """One CSV line in the olaf_c query format (fingerprint.py:276-277)."""
    return (f"{m.match_count}, {m.query_start:.4f}, {m.query_stop:.4f}, {m.reference_path}, {m.reference_id}, "
            f"{m.reference_start:.4f}, {m.reference_stop:.4f}")


# ---------------------------------------------------------------- engine-backed service

def db_path() -> Path:
    return Path(os.environ.get("AIDFP_DB") or os.environ.get("OLAF_DB") or DEFAULT_DB)


class FingerprintService:
    """One GPU engine + the persisted index of the OLAF_DB directory."""

    def __init__(self, db_dir: Path | None = None, device: int = -1):
        self.db_dir = Path(db_dir) if db_dir is not None else db_path()
        self.device = device
        self._lock = threading.Lock()
        self._engine = None
        self._ids: dict[str, int] = {}  # uuid string -> engine track id
        self._names: dict[int, str] = {}
        self._next = 0
        self.persist = True

    # -- engine and persistence --
    def _eng(self):
        if self._engine is None:
            from ._lib import EngineError, EngineUnavailable
            from .engine import Engine

            try:
                self._engine = Engine(SAMPLE_RATE, device=self.device)
            except (EngineUnavailable, EngineError, OSError) as exc:
                raise OlafError(f"fingerprint engine binary not found or unusable (libaidfp.so): {exc}") from exc
            self._load()
        return self._engine

    def _load(self) -> None:
        idx, meta = self.db_dir / "index.aidfp", self.db_dir / "tracks.json"
        if idx.exists() and meta.exists():
            self._engine.index_load(str(idx))
            d = json.loads(meta.read_text())
            self._ids = {k: int(v) for k, v in d["ids"].items()}
            self._names = {v: k for k, v in self._ids.items()}
            self._next = int(d["next"])

    def _save(self) -> None:
        if not self.persist:
            return
        self.db_dir.mkdir(parents=True, exist_ok=True)
        tmp = self.db_dir / "index.aidfp.tmp"
        self._engine.index_save(str(tmp))
        os.replace(tmp, self.db_dir / "index.aidfp")
        (self.db_dir / "tracks.json.tmp").write_text(json.dumps({"ids": self._ids, "next": self._next}))
        os.replace(self.db_dir / "tracks.json.tmp", self.db_dir / "tracks.json")

    @staticmethod
    def _pcm(buf: bytes) -> np.ndarray:
        return np.frombuffer(buf[: len(buf) // 4 * 4], dtype="<f4").astype(np.float32)

    # -- operations (blocking; call from a worker thread) --
    def index_track(self, pcm: bytes, name: str) -> bool:
        from ._lib import EngineError

        with self._lock:
            eng = self._eng()
            try:
                recs = eng.extract_host([self._pcm(pcm)])[0]
                old = self._ids.get(name)
                if old is not None:  # re-store replaces the previous fingerprints
                    eng.index_remove(old)
                    self._names.pop(old, None)
                tid = self._next
                self._next += 1
                eng.index_add_records(tid, recs)
                self._ids[name] = tid
                self._names[tid] = name
                self._save()
                return True
            except EngineError as exc:
                logger.error("aidfp store failed for %s: %s", name, exc)
                return False

    def query(self, pcm: bytes) -> list[OlafMatch]:
        from ._lib import EngineError

        with self._lock:
            eng = self._eng()
            try:
                eng.extract_host([self._pcm(pcm)])
                rows = eng.query_extracted()[0]
            except EngineError as exc:
                logger.error("aidfp query failed: %s", exc)
                return []
            sec = eng.hop / eng.sample_rate
            out = []
            for count, track, d, tq0, tq1 in rows.tolist():
                name = self._names.get(int(track))
                if name is None:
                    continue
                out.append(OlafMatch(int(count), tq0 * sec, tq1 * sec, name, int(track), (tq0 + d) * sec,
                                     (tq1 + d) * sec))
            out.sort(key=lambda m: m.match_count, reverse=True)
            return out

    def exact_batch(self, clips: list[bytes], max_results: int) -> list[list]:
        """Batched exact lane over the engine (aid_exact_lane); ranked ScoredCandidate lists."""
        from ._lib import EngineError
        from .exact import candidates_from_rows

        with self._lock:
            eng = self._eng()
            pcms = [self._pcm(c) for c in clips]
            try:
                rows = eng.exact_lane(pcms)
            except EngineError as exc:
                logger.error("aidfp exact lane failed: %s", exc)
                return [[] for _ in clips]
            return [candidates_from_rows(r, self._names, max_results) if len(p) else []
                    for r, p in zip(rows, pcms)]

    def delete_track(self, name: str) -> bool:
        from ._lib import EngineError

        with self._lock:
            eng = self._eng()
            tid = self._ids.get(name)
            if tid is None:
                logger.error("aidfp del: unknown track %s", name)
                return False
            try:
                eng.index_remove(tid)
            except EngineError as exc:
                logger.error("aidfp del failed for %s: %s", name, exc)
                return False
            del self._ids[name]
            self._names.pop(tid, None)
            self._save()
            return True

    def close(self) -> None:
        with self._lock:
            if self._engine is not None:
                self._engine.close()
                self._engine = None


_service: FingerprintService | None = None
_service_lock = threading.Lock()


def get_service() -> FingerprintService:
    global _service
    with _service_lock:
        if _service is None:
            _service = FingerprintService()
        return _service


def set_service(svc: FingerprintService | None) -> None:
    global _service
    with _service_lock:
        _service = svc


async def _run(fn, *args):
    return await asyncio.get_running_loop().run_in_executor(None, fn, *args)


# ---------------------------------------------------------------- reference API

async def olaf_index_track(pcm_16k_f32le: bytes, track_id: uuid.UUID) -> bool:
    if not pcm_16k_f32le:
        logger.warning("empty PCM for track %s", track_id)
        return False
    try:
        return await _run(get_service().index_track, pcm_16k_f32le, str(track_id))
    except OlafError:
        raise
    except Exception as exc:
        logger.exception("unexpected error indexing %s", track_id)
        raise OlafError(f"Failed to index track {track_id}: {exc}") from exc


async def olaf_query(pcm_16k_f32le: bytes) -> list[OlafMatch]:
    if not pcm_16k_f32le:
        return []
    try:
        return await _run(get_service().query, pcm_16k_f32le)
    except OlafError:
        raise
    except Exception as exc:
        logger.exception("unexpected error during query")
        raise OlafError(f"Failed to query: {exc}") from exc


async def olaf_delete_track(track_id: uuid.UUID) -> bool:
    try:
        return await _run(get_service().delete_track, str(track_id))
    except OlafError:
        raise
    except Exception as exc:
        logger.exception("unexpected error deleting %s", track_id)
        raise OlafError(f"Failed to delete track {track_id}: {exc}") from exc
