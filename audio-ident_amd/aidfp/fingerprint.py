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
  OLAF_DB dir (:71-84)                        same dir: snapshot + journal (aidfp.store)

Error contract (reference :102-155, :173-219, :234-270):
  * empty PCM -> False / [] without touching the engine;
  * engine cannot load (no libaidfp.so / no gfx950 GPU) -> OlafError whose message
    says the fingerprint engine binary was not found;
  * a recoverable engine error (bad input, unknown track on delete) -> False / []
    (logged), like a non-zero olaf_c exit code;
  * anything unexpected -> OlafError.
Concurrency (aidfp.concurrency): index writes take a reader/writer lock exclusively
(the reference's LMDB single-writer rule, :7-8); queries share it. Concurrent
olaf_query calls -- the reference runs one `olaf_c query` process each (:185-193)
-- are coalesced into one engine call (aid_query_pcm) by a dispatcher thread, and
the coroutine awaits its own future, so the event loop is never blocked. Writes run
in a worker thread (ctypes releases the GIL).
"""

from __future__ import annotations

import asyncio
import logging
import os
import threading
import time
import uuid
from dataclasses import dataclass
from pathlib import Path

import numpy as np

from .concurrency import QueryCoalescer, RWLock

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


class _Answered:
    """A coalesced batch answered at submit time (its engine submit failed and the synchronous path ran)."""

    __slots__ = ("out",)

    def __init__(self, out):
        self.out = out

    def collect(self):
        return self.out


class _PendingBatch:
    """A coalesced batch in flight: holds the service's shared lock from submit until collect()."""

    __slots__ = ("svc", "eng", "pcms", "pend")

    def __init__(self, svc, eng, pcms, pend):
        self.svc, self.eng, self.pcms, self.pend = svc, eng, pcms, pend

    def collect(self):
        from ._lib import EngineError

        try:
            try:
                rows = self.pend.collect()
            except EngineError as exc:
                rows = self.svc._rows_after_failure(self.eng, self.pcms, exc)
            return self.svc._matches(self.eng, rows)
        finally:
            self.svc._rw.release_read()


class FingerprintService:
    """One GPU engine + the persisted index of the OLAF_DB directory (aidfp.store: snapshot +
    write-ahead journal, so a store or delete writes O(track) bytes, not the whole index)."""

    def __init__(self, db_dir: Path | None = None, device: int = -1, checkpoint_min_bytes: int = 64 << 20,
                 coalesce_window_s: float | None = None, max_batch: int = 256, max_batch_bytes: int = 64 << 20,
                 coalesce_workers: int = 1, pipeline: bool = True, split_min: int = 16, split_parts: int = 2):
        self.db_dir = Path(db_dir) if db_dir is not None else db_path()
        self.device = device
        self._rw = RWLock()  # index writers exclusive, queries shared
        self._init_lock = threading.Lock()  # first-use engine creation + index load
        # a coalesced batch holds at most max_batch requests and max_batch_bytes of PCM (64 MiB = 17 min of
        # 16 kHz audio): many long uploads cannot land in one extraction
        # pipeline: the coalescer starts batch N + 1 (aid_query_pcm_submit) before it collects batch N. The next
        # batch then gathers while the current one is in flight, so a pipelined coalescer waits for no window:
        # 40-45 k qps at 64 clients and 27 k at 16 with none, against 30-34 k and 14 k with 0.5 ms
        # (profiles/r06akl_service_window_ab.jsonl); the one-call path keeps its 0.5 ms window
        if coalesce_window_s is None:  # (the coalescer pipelines with one dispatcher thread only)
            coalesce_window_s = 0.0 if pipeline and coalesce_workers == 1 else 0.0005
        self._coalescer = QueryCoalescer(self._query_batch, coalesce_window_s, max_batch, max_batch_bytes,
                                         coalesce_workers, self._submit_batch if pipeline else None, split_min,
                                         split_parts)
        self._ckpt_retry_at = 0.0  # monotonic time before which a failed auto-checkpoint is not retried
        self._engine = None
        self._store = None
        self._ids: dict[str, int] = {}  # uuid string -> engine track id
        self._names: dict[int, str] = {}
        self._next = 0
        # persist = False: stores and deletes skip the journal and the automatic checkpoints (bulk
        # ingest); the catalog on disk is still loaded first, and checkpoint() writes everything
        self.persist = True
        self.checkpoint_min_bytes = checkpoint_min_bytes
        from .engine import on_shutdown

        on_shutdown(self)  # closed (coalescer thread joined, engine destroyed) at exit, before the HIP runtime goes

    # -- engine and persistence --
    def _eng(self):
        """The engine, created and loaded from the OLAF_DB directory on first use. The service
        keeps it only once the saved index has been loaded completely: a failed load destroys
        the engine and raises OlafError, so nothing is ever written over a catalog that was not
        read (the next call retries the load)."""
        if self._engine is not None:
            return self._engine
        with self._init_lock:
            return self._eng_locked()

    def _eng_locked(self):
        if self._engine is None:
            from ._lib import EngineError, EngineUnavailable
            from .engine import Engine
            from .store import OP_STORE, IndexStore, StoreCorrupt

            try:
                eng = Engine(SAMPLE_RATE, device=self.device)
            except (EngineUnavailable, EngineError, OSError) as exc:
                raise OlafError(f"fingerprint engine binary not found or unusable (libaidfp.so): {exc}") from exc
            store = IndexStore(self.db_dir, self.checkpoint_min_bytes)
            ids: dict[str, int] = {}
            names: dict[int, str] = {}
            try:
                ids, nxt, entries = store.load(eng)
                names = {v: k for k, v in ids.items()}
                for op, track, name, recs in entries:  # replay the journal in order
                    if op == OP_STORE:
                        self._apply_store(eng, ids, names, track, name, recs)
                    else:
                        self._apply_delete(eng, ids, names, track, name)
            except (EngineError, StoreCorrupt, OSError) as exc:
                eng.close()
                raise OlafError(f"cannot load the fingerprint index in {self.db_dir}: {exc}") from exc
            except BaseException:
                eng.close()
                raise
            # the maps first, the engine last: _eng()'s lock-free fast path returns as soon as _engine is set,
            # and a reader that got it must find the names of the loaded tracks
            self._ids, self._names, self._next, self._store = ids, names, nxt, store
            self._engine = eng
        return self._engine

    @staticmethod
    def _apply_store(eng, ids, names, track: int, name: str, recs) -> None:
        """A store of `name` as `track` (the journal's replay and the live path do the same)."""
        eng.index_add_records(track, recs)
        old = ids.get(name)
        if old is not None and old != track:  # re-store replaces the previous fingerprints
            FingerprintService._remove_quiet(eng, old)
            names.pop(old, None)
        ids[name] = track
        names[track] = name

    @staticmethod
    def _remove_quiet(eng, track: int) -> None:
        """Replay: an id without an engine slot (a zero-hash track of an older index) has nothing
        to remove."""
        from ._lib import EngineError

        try:
            eng.index_remove(track)
        except EngineError as exc:
            logger.warning("aidfp journal replay: remove of track %d: %s", track, exc)

    @staticmethod
    def _apply_delete(eng, ids, names, track: int, name: str) -> None:
        FingerprintService._remove_quiet(eng, track)
        if ids.get(name) == track:
            del ids[name]
        names.pop(track, None)

    def _maybe_checkpoint(self) -> None:
        """Automatic checkpoint after a write. The operation is already journaled (fsynced) and applied,
        so a failed checkpoint (full disk, permissions, device error in the compaction) is logged and
        the journal kept -- the caller still gets True -- and retried no sooner than 60 s later."""
        from ._lib import EngineError

        if not (self.persist and self._store.should_checkpoint()) or time.monotonic() < self._ckpt_retry_at:
            return
        try:
            self._store.checkpoint(self._engine, dict(self._ids), self._next)
        except (OSError, EngineError):  # the journal still holds every operation: nothing is lost
            logger.exception("aidfp index checkpoint failed (journal kept)")
            self._ckpt_retry_at = time.monotonic() + 60.0
            for tmp in self.db_dir.glob("*.tmp"):
                tmp.unlink(missing_ok=True)

    @staticmethod
    def _pcm(buf: bytes) -> np.ndarray:
        # a read-only float32 view of the request bytes (no copy; the engine call copies once into its batch)
        return np.frombuffer(buf, dtype="<f4", count=len(buf) // 4).astype(np.float32, copy=False)

    # -- operations (blocking; call from a worker thread) --
    def index_track(self, pcm: bytes, name: str) -> bool:
        from ._lib import EngineError

        with self._rw.write():
            eng = self._eng()
            try:
                recs = eng.extract_host([self._pcm(pcm)])[0]
                tid = self._next
                # the new postings first, the journal entry, then the old ones go: a failed
                # append leaves the previous fingerprints of `name` live
                eng.index_add_records(tid, recs)
                self._next += 1
            except EngineError as exc:
                logger.error("aidfp store failed for %s: %s", name, exc)
                return False
            if self.persist:
                try:
                    self._store.append_store(tid, name, recs)
                except OSError as exc:
                    logger.error("aidfp store of %s not persisted: %s", name, exc)
                    eng.index_remove(tid)
                    return False
            try:
                self._apply_store_maps(eng, name, tid)
            except EngineError as exc:
                logger.error("aidfp store of %s: removing the previous fingerprints failed: %s", name, exc)
            self._maybe_checkpoint()
            return True

    def _apply_store_maps(self, eng, name: str, tid: int) -> None:
        old = self._ids.get(name)
        self._ids[name] = tid
        self._names[tid] = name
        if old is not None and old != tid:
            self._names.pop(old, None)
            eng.index_remove(old)

    def register_tracks(self, names: dict) -> None:
        """Name the engine track ids of postings that were added to this service's engine directly (a bulk
        catalog built on the device, e.g. aidfp.catalog.ingest_synthetic): `names` maps name -> track id, as
        index_track records per store. Not journaled: call checkpoint() to persist (the bulk-ingest recipe)."""
        with self._rw.write():
            self._eng()
            for name, tid in names.items():
                self._ids[str(name)] = int(tid)
                self._names[int(tid)] = str(name)
            self._next = max([self._next] + [int(t) + 1 for t in names.values()])

    def submit_query(self, pcm: bytes):
        """Queue one query for the coalescer; returns a concurrent.futures.Future of list[OlafMatch]."""
        return self._coalescer.submit(pcm)

    def submit_query_async(self, pcm: bytes):
        """Queue one query from a running event loop; returns an asyncio future of list[OlafMatch]."""
        return self._coalescer.submit_async(pcm)

    def query(self, pcm: bytes) -> list[OlafMatch]:
        return self._coalescer(pcm)

    def _query_rows(self, eng, pcms: list[bytes]) -> list:
        """Engine rows per request. If the batch's engine call fails in a way that depends on the batch (one
        request's vote table overflows: AID_ERR_STATE; a large batch runs out of memory: AID_ERR_NOMEM), the
        batch is bisected and retried, so only the request that fails on its own gets [] -- like one failing
        `olaf_c query` process (fingerprint.py:197-200). A device fault or an invalid argument does not depend
        on the batch: the whole batch gets [] at once (bisecting a sticky device fault would cost ~2n failing
        engine calls under the shared lock)."""
        from ._lib import EngineError

        try:
            return eng.query_pcm([self._pcm(p) for p in pcms])
        except EngineError as exc:
            return self._rows_after_failure(eng, pcms, exc)

    def _rows_after_failure(self, eng, pcms: list[bytes], exc) -> list:
        """The batch's engine call (or its pipelined submit / collect) failed with `exc`: [] for every request, or
        the batch bisected and retried if the failure depends on the batch (see _query_rows)."""
        from ._lib import AID_ERR_NOMEM, AID_ERR_STATE

        if len(pcms) == 1 or exc.code not in (AID_ERR_STATE, AID_ERR_NOMEM):
            logger.error("aidfp query batch of %d failed: %s", len(pcms), exc)
            return [np.zeros((0, 5), np.int64) for _ in pcms]
        logger.warning("aidfp query batch of %d failed (%s); retrying in halves", len(pcms), exc)
        h = len(pcms) // 2
        return self._query_rows(eng, pcms[:h]) + self._query_rows(eng, pcms[h:])

    def _matches(self, eng, rows) -> list[list[OlafMatch]]:
        """Engine rows -> OlafMatch lists (under the shared lock: the name map is the index's)."""
        sec = eng.hop / eng.sample_rate
        outs = []
        for r in rows:
            out = []
            for count, track, d, tq0, tq1 in r.tolist():
                name = self._names.get(int(track))
                if name is None:
                    continue
                out.append(OlafMatch(int(count), tq0 * sec, tq1 * sec, name, int(track), (tq0 + d) * sec,
                                     (tq1 + d) * sec))
            out.sort(key=lambda m: m.match_count, reverse=True)
            outs.append(out)
        return outs

    def _query_batch(self, pcms: list[bytes]) -> list[list[OlafMatch]]:
        """One engine call for every query the coalescer gathered (under the shared lock)."""
        with self._rw.read():
            eng = self._eng()
            return self._matches(eng, self._query_rows(eng, pcms))

    def _submit_batch(self, pcms: list[bytes], behind: bool):
        """The coalescer's pipelined half: take the shared lock, queue the batch (aid_query_pcm_submit) and return
        a handle whose collect() answers it and releases the lock. With a batch still outstanding (`behind`) the
        lock is taken only if no writer waits for it (else None: the coalescer finishes that batch first)."""
        from ._lib import EngineError

        if behind:
            if not self._rw.try_acquire_read():
                return None
        else:
            self._rw.acquire_read()
        try:
            eng = self._eng()
            try:
                return _PendingBatch(self, eng, pcms, eng.query_pcm_submit([self._pcm(p) for p in pcms]))
            except EngineError as exc:  # answered now (bisecting a batch-dependent failure)
                out = self._matches(eng, self._rows_after_failure(eng, pcms, exc))
        except BaseException:
            self._rw.release_read()
            raise
        self._rw.release_read()
        return _Answered(out)

    def exact_batch(self, clips: list[bytes], max_results: int) -> list[list]:
        """Batched exact lane over the engine (aid_exact_lane); ranked ScoredCandidate lists."""
        from ._lib import EngineError
        from .exact import candidates_from_rows

        with self._rw.read():
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

        with self._rw.write():
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
            if self.persist:
                try:
                    self._store.append_delete(tid, name)
                except OSError as exc:  # removed now, but it comes back after a restart
                    logger.error("aidfp del of %s not persisted: %s", name, exc)
                    return False
            self._maybe_checkpoint()
            return True

    def checkpoint(self) -> None:
        """Write a snapshot of the whole index now (compacting removed tracks' postings) and start an
        empty journal. Always writes, also with persist = False: that is how a bulk ingest commits."""
        with self._rw.write():
            self._eng()
            self._store.checkpoint(self._engine, dict(self._ids), self._next)

    def close(self) -> None:
        self._coalescer.close()
        with self._rw.write():
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
        # coalesced with the other queries in flight (one engine call per batch); no worker thread waits, and the
        # batch's results reach this loop in one callback
        return await get_service().submit_query_async(pcm_16k_f32le)
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
