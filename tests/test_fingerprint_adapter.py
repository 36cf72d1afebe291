"""Error contract and persistence of the drop-in aidfp.fingerprint module, in the
style of the reference's tests/test_audio_fingerprint.py (which mocks the olaf_c
subprocess): here the GPU engine class is replaced by a small test double so the
host logic runs without a GPU. The real engine path is covered by
tests/test_gpu_adapter.py."""

import asyncio
import json
import os
import uuid

import numpy as np
import pytest

from aidfp import _lib
from aidfp import cli
from aidfp import fingerprint as fp

TID = uuid.UUID("12345678-1234-5678-1234-567812345678")
PCM = np.arange(4000, dtype="<f4").tobytes()


class FakeEngine:
    """Test double of aidfp.engine.Engine: 'fingerprints' are the first PCM values, carried in
    the records (so a journal replay restores them); save/load keep the live state as JSON."""

    fail_load = False  # class-wide: the next engine's index_load raises (truncated file, OOM ...)
    saved_bytes = 0    # bytes written by index_save, all engines

    def __init__(self, sample_rate, device=-1, fail=None):
        self.sample_rate, self.hop = sample_rate, 256
        self.tracks, self.removed, self.fail = {}, set(), fail
        self.closed = False

    def extract_host(self, clips):
        if self.fail == "extract":
            raise _lib.EngineError(-1, "bad input")
        self._last = [np.asarray(c[:3], dtype=np.float32) for c in clips]
        return [np.asarray(c[:3], dtype=np.float32).view(np.uint32).astype(np.uint64) for c in clips]

    def index_add_records(self, track, recs):
        self.tracks[track] = np.asarray(recs, dtype=np.uint64).astype(np.uint32).view(np.float32)

    def index_compact(self):
        n = sum(len(self.tracks.pop(t)) for t in list(self.removed) if t in self.tracks)
        return n

    def index_remove(self, track):
        if track in self.removed or track not in self.tracks:
            raise _lib.EngineError(-1, "track not indexed")
        self.removed.add(track)

    def query_extracted(self):
        q = self._last[0]
        rows = [[10 + t, t, 4, 1, 20] for t, v in self.tracks.items() if t not in self.removed and np.array_equal(v, q)]
        rows += [[5, t, 0, 0, 2] for t in self.tracks if t not in self.removed and len(rows) < 3]
        return [np.array(rows, dtype=np.int64).reshape(-1, 5)]

    def query_pcm(self, clips):
        if self.fail == "extract":
            raise _lib.EngineError(-1, "bad input")
        out = []
        for c in clips:
            self._last = [np.asarray(c[:3], dtype=np.float32)]
            out.append(self.query_extracted()[0])
        return out

    def query_pcm_submit(self, clips):  # the coalescer's pipelined half: answered at submit, handed back at collect
        out = self.query_pcm(clips)
        self.submits = getattr(self, "submits", 0) + 1
        return type("Pending", (), {"collect": lambda _self: out})()

    def index_save(self, path):
        blob = json.dumps({"tracks": {str(t): v.tolist() for t, v in self.tracks.items()},
                           "removed": sorted(self.removed)})
        open(path, "w").write(blob)
        FakeEngine.saved_bytes += len(blob)

    def index_load(self, path):
        if FakeEngine.fail_load:
            raise _lib.EngineError(-2, "truncated index file")
        d = json.loads(open(path).read())
        self.tracks = {int(t): np.asarray(v, dtype=np.float32) for t, v in d["tracks"].items()}
        self.removed = set(d["removed"])

    def close(self):
        self.closed = True


@pytest.fixture
def svc(tmp_path, monkeypatch):
    import aidfp.engine as E

    monkeypatch.setattr(E, "Engine", FakeEngine)
    s = fp.FingerprintService(tmp_path / "db")
    fp.set_service(s)
    yield s
    fp.set_service(None)


def run(c):
    return asyncio.run(c)


def test_index_empty_pcm_returns_false(svc):
    assert run(fp.olaf_index_track(b"", TID)) is False
    assert svc._engine is None  # engine never touched


def test_index_success_persists(svc, tmp_path):
    assert run(fp.olaf_index_track(PCM, TID)) is True
    assert (tmp_path / "db" / "journal.0.aidfj").exists()  # one journal entry, no full rewrite
    again = fp.FingerprintService(tmp_path / "db")  # a restart replays it
    assert again.query(PCM)[0].reference_path == str(TID)


def test_index_engine_error_returns_false(svc):
    svc._eng().fail = "extract"
    assert run(fp.olaf_index_track(PCM, TID)) is False
    assert run(fp.olaf_query(PCM)) == []


def test_engine_unavailable_raises(tmp_path, monkeypatch):
    import aidfp.engine as E

    def boom(*a, **k):
        raise _lib.EngineUnavailable("libaidfp.so missing")

    monkeypatch.setattr(E, "Engine", boom)
    fp.set_service(fp.FingerprintService(tmp_path))
    try:
        for coro in (fp.olaf_index_track(PCM, TID), fp.olaf_query(PCM), fp.olaf_delete_track(TID)):
            with pytest.raises(fp.OlafError, match="binary not found"):
                run(coro)
    finally:
        fp.set_service(None)


def test_unexpected_error_wrapped(svc, monkeypatch):
    monkeypatch.setattr(svc, "index_track", lambda *a: (_ for _ in ()).throw(RuntimeError("disk on fire")))
    with pytest.raises(fp.OlafError, match="Failed to index track"):
        run(fp.olaf_index_track(PCM, TID))


def test_query_rows_sorted_and_mapped(svc):
    other = uuid.UUID(int=7)
    assert run(fp.olaf_index_track(PCM, TID))
    assert run(fp.olaf_index_track(np.ones(100, "<f4").tobytes(), other))
    res = run(fp.olaf_query(PCM))
    assert [m.match_count for m in res] == sorted((m.match_count for m in res), reverse=True)
    top = res[0]
    assert top.reference_path == str(TID) and top.match_count == 10
    sec = 256 / 16000
    assert top.query_start == pytest.approx(1 * sec) and top.query_stop == pytest.approx(20 * sec)
    assert top.reference_start == pytest.approx(5 * sec) and top.reference_stop == pytest.approx(24 * sec)
    assert run(fp.olaf_query(b"")) == []


def test_delete_and_restore(svc):
    assert run(fp.olaf_delete_track(TID)) is False  # unknown -> like a non-zero olaf_c exit
    assert run(fp.olaf_index_track(PCM, TID))
    assert run(fp.olaf_delete_track(TID)) is True
    assert all(m.reference_path != str(TID) for m in run(fp.olaf_query(PCM)))
    assert run(fp.olaf_index_track(PCM, TID))  # re-store after delete
    assert run(fp.olaf_query(PCM))[0].reference_path == str(TID)
    assert run(fp.olaf_index_track(PCM, TID))  # re-store replaces: still one live id
    assert len(svc._ids) == 1


def test_cli_shim_roundtrip(tmp_path, monkeypatch, capsys):
    import aidfp.engine as E

    monkeypatch.setattr(E, "Engine", FakeEngine)
    monkeypatch.setenv("OLAF_DB", str(tmp_path / "clidb"))
    raw = tmp_path / "q.raw"
    raw.write_bytes(PCM)
    assert cli.main(["store", str(raw), str(TID)]) == 0
    assert cli.main(["query", str(raw), "query"]) == 0
    out = capsys.readouterr().out
    parsed = fp._parse_olaf_output(out)
    assert isinstance(parsed, list)
    assert cli.main(["del", "not-there"]) == 1
    assert cli.main(["bogus"]) == 2


# ---------------------------------------------------------------- persistence (aidfp.store)

def _svc(path, **kw):
    return fp.FingerprintService(path, **kw)


@pytest.fixture
def fake_engine(monkeypatch):
    import aidfp.engine as E

    monkeypatch.setattr(E, "Engine", FakeEngine)
    FakeEngine.fail_load = False
    FakeEngine.saved_bytes = 0
    yield FakeEngine
    FakeEngine.fail_load = False


def _pcm(i):
    return np.array([i, i + 0.5, -i, 7], dtype="<f4").tobytes()


def test_failed_load_never_overwrites_the_catalog(fake_engine, tmp_path):
    """a failed index load must not let the next store replace the saved catalog."""
    db = tmp_path / "db"
    s = _svc(db, checkpoint_min_bytes=0)  # checkpoint on every write: a snapshot exists
    a, b, c = (str(uuid.UUID(int=i)) for i in (1, 2, 3))
    assert s.index_track(_pcm(1), a) and s.index_track(_pcm(2), b)
    s.close()
    before = {p.name: p.read_bytes() for p in db.iterdir()}
    fake_engine.fail_load = True
    s2 = _svc(db, checkpoint_min_bytes=0)
    with pytest.raises(fp.OlafError, match="cannot load"):
        s2.index_track(_pcm(3), c)
    assert s2._engine is None
    with pytest.raises(fp.OlafError):  # every later call retries the load, none writes
        s2.delete_track(a)
    assert {p.name: p.read_bytes() for p in db.iterdir()} == before
    fake_engine.fail_load = False
    assert s2.index_track(_pcm(3), c)  # the load succeeds now: the catalog is {a, b, c}
    s3 = _svc(db)
    s3._eng()
    assert sorted(s3._ids) == sorted([a, b, c])


def test_journal_replay_restores_stores_and_deletes(fake_engine, tmp_path):
    db = tmp_path / "db"
    s = _svc(db)
    names = [str(uuid.UUID(int=i)) for i in range(6)]
    for i, n in enumerate(names):
        assert s.index_track(_pcm(i), n)
    assert s.delete_track(names[1])
    assert s.index_track(_pcm(40), names[2])  # re-store replaces
    ids, nxt = dict(s._ids), s._next
    s.close()
    r = _svc(db)
    r._eng()
    assert r._ids == ids and r._next == nxt
    assert r.query(_pcm(40))[0].reference_path == names[2]
    assert all(m.reference_path != names[1] for m in r.query(_pcm(1)))


def test_torn_journal_tail_is_dropped(fake_engine, tmp_path):
    db = tmp_path / "db"
    s = _svc(db)
    assert s.index_track(_pcm(1), "a") and s.index_track(_pcm(2), "b")
    s.close()
    j = db / "journal.0.aidfj"
    good = j.stat().st_size
    with open(j, "ab") as f:  # a crash in the middle of a third append
        f.write(b"AIDJ\x01\x00\x00\x00garbage")
    r = _svc(db)
    r._eng()
    assert sorted(r._ids) == ["a", "b"]
    assert j.stat().st_size == good
    assert r.index_track(_pcm(3), "c")  # appends continue after the repaired tail
    r2 = _svc(db)
    r2._eng()
    assert sorted(r2._ids) == ["a", "b", "c"]


def test_checkpoint_compacts_and_crash_keeps_old_generation(fake_engine, tmp_path, monkeypatch):
    db = tmp_path / "db"
    s = _svc(db, checkpoint_min_bytes=1 << 30)
    for i in range(4):
        assert s.index_track(_pcm(i), f"t{i}")
    assert s.delete_track("t0")
    s.checkpoint()
    assert json.loads((db / "tracks.json").read_text())["gen"] == 1
    assert 0 not in s._engine.tracks  # removed postings compacted before the snapshot
    assert not (db / "journal.0.aidfj").exists()
    assert s.index_track(_pcm(9), "t9")
    # a crash inside the next checkpoint, after the snapshot write, before the manifest commit
    real_replace = os.replace

    def crash(src, dst):
        if str(dst).endswith("tracks.json"):
            raise OSError("power cut")
        return real_replace(src, dst)

    monkeypatch.setattr(os, "replace", crash)
    with pytest.raises(OSError):
        s.checkpoint()
    monkeypatch.setattr(os, "replace", real_replace)
    r = _svc(db)
    r._eng()
    assert sorted(r._ids) == ["t1", "t2", "t3", "t9"]  # generation 1 + its journal


def test_ingest_bytes_grow_linearly(fake_engine, tmp_path):
    """N stores must not rewrite the whole index each time (O(N^2) bytes)."""
    db = tmp_path / "db"
    s = _svc(db, checkpoint_min_bytes=4096)
    n = 400
    for i in range(n):
        assert s.index_track(_pcm(i), f"track-{i}")
    journal = s._store.journal_bytes
    snap_bytes = FakeEngine.saved_bytes
    final = (db / s._store.snapshot).stat().st_size if s._store.snapshot else 0
    # every checkpoint at least doubles the bytes it folds in: snapshots total < 2x the final one
    assert snap_bytes <= 2 * final + 4096
    assert journal <= max(4096, final) + 200
    r = _svc(db)
    r._eng()
    assert len(r._ids) == n


def test_zero_hash_track_delete_and_restore(fake_engine, tmp_path):
    """a clip with no hashes still gets an id that can be deleted and re-stored."""
    s = _svc(tmp_path / "db")
    short = np.zeros(0, dtype="<f4").tobytes() + np.zeros(1, dtype="<f4").tobytes()
    assert s.index_track(short, "tiny")
    assert s.delete_track("tiny")
    assert s.index_track(short, "tiny") and s.index_track(short, "tiny")


def test_exact_lane_engine_unavailable_returns_empty(tmp_path, monkeypatch):
    """the reference's exact lane logs an OlafError and returns [] (exact.py:163-171)."""
    import aidfp.engine as E
    from aidfp import exact

    def boom(*a, **k):
        raise _lib.EngineUnavailable("libaidfp.so missing")

    monkeypatch.setattr(E, "Engine", boom)
    fp.set_service(fp.FingerprintService(tmp_path))
    try:
        got = run(exact.run_exact_lane_batch([PCM, PCM], 5, lookup=lambda ids: {}))
        assert got == [[], []]
        assert run(exact.run_exact_lane(PCM, 5)) == []
    finally:
        fp.set_service(None)


def _pcm_of(v: float) -> bytes:
    return np.full(16000, v, dtype="<f4").tobytes()


def test_concurrent_queries_coalesced_equal_serial(svc, monkeypatch):
    """64 concurrent olaf_query coroutines (the reference would spawn 64 olaf_c processes) are served by
    a few batched engine calls and each gets exactly the rows of a serial call with its PCM."""
    import time as _t

    names = [uuid.UUID(int=1000 + i) for i in range(8)]
    for i, n in enumerate(names):
        assert run(fp.olaf_index_track(_pcm_of(0.1 * (i + 1)), n))
    serial = {i: svc.query(_pcm_of(0.1 * (i % 8 + 1))) for i in range(8)}
    eng = svc._eng()
    slow = eng.query_pcm
    calls = []

    def slow_query(clips):  # a batch takes 5 ms: later arrivals queue up behind it
        calls.append(len(clips))
        _t.sleep(0.005)
        return slow(clips)

    monkeypatch.setattr(eng, "query_pcm", slow_query)

    async def many():
        return await asyncio.gather(*[fp.olaf_query(_pcm_of(0.1 * (i % 8 + 1))) for i in range(64)])

    got = run(many())
    for i, rows in enumerate(got):
        assert rows == serial[i % 8]
        assert rows and rows[0].reference_path == str(names[i % 8])
    assert sum(calls) == 64 and len(calls) < 64 and max(calls) > 1


def test_queries_wait_for_writer(svc):
    """A query submitted while a store holds the write lock runs after it and sees the new track."""
    import threading

    tid = uuid.UUID(int=77)
    svc._eng()
    svc._rw.acquire_write()
    fut = svc.submit_query(_pcm_of(0.5))
    t = threading.Thread(target=lambda: None)
    t.start()
    t.join()
    assert not fut.done()
    # the writer's work, done while holding the lock (index_track would take it itself)
    eng = svc._engine
    recs = eng.extract_host([np.full(16000, 0.5, np.float32)])[0]
    eng.index_add_records(svc._next, recs)
    svc._apply_store_maps(eng, str(tid), svc._next)
    svc._next += 1
    svc._rw.release_write()
    assert fut.result(timeout=10)[0].reference_path == str(tid)


def test_bulk_ingest_recipe(svc, tmp_path):
    """INTEGRATION.md bulk ingest: persist = False skips the per-track journal, the catalog already on
    disk is still loaded first, and one checkpoint() commits everything for the next start."""
    first = uuid.UUID(int=1)
    assert run(fp.olaf_index_track(_pcm_of(0.9), first))  # an existing catalog (journaled)
    bulk = fp.FingerprintService(tmp_path / "db")
    bulk.persist = False
    names = [uuid.UUID(int=10 + i) for i in range(5)]
    for i, n in enumerate(names):
        assert bulk.index_track(_pcm_of(0.2 + 0.1 * i), str(n))
    jour = tmp_path / "db" / "journal.0.aidfj"
    size_before = jour.stat().st_size
    assert jour.stat().st_size == size_before  # nothing journaled during the bulk
    bulk.checkpoint()
    bulk.close()
    again = fp.FingerprintService(tmp_path / "db")
    assert again.query(_pcm_of(0.9))[0].reference_path == str(first)
    for i, n in enumerate(names):
        assert again.query(_pcm_of(0.2 + 0.1 * i))[0].reference_path == str(n)


def test_failed_auto_checkpoint_keeps_operation(svc, tmp_path, monkeypatch):
    """A checkpoint that fails inside the engine (EngineError) after the store was journaled leaves the
    store successful (True), removes the half-written snapshot and keeps the journal for the restart."""
    svc.checkpoint_min_bytes = 1
    svc._eng()
    svc._store.checkpoint_min_bytes = 1
    eng = svc._engine

    def bad_save(path):
        open(path, "w").write("partial")
        raise _lib.EngineError(-2, "device error while saving")

    monkeypatch.setattr(eng, "index_save", bad_save)
    tid = uuid.UUID(int=5)
    assert run(fp.olaf_index_track(_pcm_of(0.3), tid)) is True
    assert not list((tmp_path / "db").glob("*.tmp"))
    assert run(fp.olaf_index_track(_pcm_of(0.4), uuid.UUID(int=6))) is True  # backoff: no retry storm
    again = fp.FingerprintService(tmp_path / "db")
    assert again.query(_pcm_of(0.3))[0].reference_path == str(tid)


def test_one_failing_request_does_not_blank_its_batch(svc, monkeypatch):
    """A coalesced batch whose engine call fails (one request overflows its vote table, AID_ERR_STATE) is
    bisected and retried: only the request that fails on its own gets [], every other request of the batch
    still gets its rows (the reference's olaf_c processes failed one by one, fingerprint.py:197-200)."""
    import time as _t

    names = [uuid.UUID(int=2000 + i) for i in range(8)]
    for i, n in enumerate(names):
        assert run(fp.olaf_index_track(_pcm_of(0.1 * (i + 1)), n))
    eng = svc._eng()
    real = eng.query_pcm
    calls = []
    poison = np.float32(0.77)

    def picky_query(clips):
        calls.append(len(clips))
        _t.sleep(0.005)  # later arrivals queue up: batches form
        if any(len(c) and c[0] == poison for c in clips):
            raise _lib.EngineError(-4, "query vote table overflow")
        return real(clips)

    monkeypatch.setattr(eng, "query_pcm", picky_query)

    async def many():
        pcms = [_pcm_of(0.1 * (i % 8 + 1)) for i in range(40)]
        pcms[17] = _pcm_of(0.77)
        return await asyncio.gather(*[fp.olaf_query(p) for p in pcms])

    got = run(many())
    assert got[17] == []
    for i, rows in enumerate(got):
        if i != 17:
            assert rows and rows[0].reference_path == str(names[i % 8]), i
    assert max(calls) > 1  # it was coalesced


def test_device_error_fails_the_batch_without_bisecting(svc, monkeypatch):
    """A device fault (AID_ERR_DEVICE) or an invalid argument does not depend on the batch: the coalesced batch
    gets [] for every request after ONE engine call, instead of ~2n bisected calls under the shared lock."""
    import time as _t

    assert run(fp.olaf_index_track(_pcm_of(0.2), uuid.UUID(int=3000)))
    eng = svc._eng()
    calls = []

    def broken(clips):
        calls.append(len(clips))
        _t.sleep(0.005)
        raise _lib.EngineError(_lib.AID_ERR_DEVICE, "hipErrorLaunchFailure")

    monkeypatch.setattr(eng, "query_pcm", broken)

    async def many():
        return await asyncio.gather(*[fp.olaf_query(_pcm_of(0.2)) for _ in range(24)])

    got = run(many())
    assert got == [[]] * 24
    assert sum(calls) == 24  # every request was sent exactly once: no retries in halves
    assert max(calls) > 1  # and the batches were coalesced


def test_coalescer_caps_batch_bytes():
    """QueryCoalescer closes a batch before the next payload would pass max_batch_bytes; that payload opens
    the next batch, and one payload above the cap runs alone."""
    import threading

    from aidfp.concurrency import QueryCoalescer

    gate = threading.Event()
    seen = []

    def runner(ps):
        gate.wait(5)
        seen.append([len(p) for p in ps])
        return [len(p) for p in ps]

    c = QueryCoalescer(runner, window_s=0.05, max_batch=64, max_batch_bytes=100)
    first = c.submit(b"x")  # the dispatcher takes it and blocks in runner until the rest are queued
    futs = [c.submit(b"y" * n) for n in (40, 40, 40, 300, 10)]
    gate.set()
    assert first.result(5) == 1
    assert [f.result(5) for f in futs] == [40, 40, 40, 300, 10]
    c.close()
    assert all(sum(b) <= 100 or len(b) == 1 for b in seen)
    assert [300] in seen


def test_register_tracks_names_a_bulk_catalog(svc, tmp_path):
    """Postings added to the service's engine directly (a device-built catalog) answer olaf_query under the names
    register_tracks gives them, new stores take the next free id, and a checkpoint persists the names."""
    eng = svc._eng()
    recs = eng.extract_host([np.full(16000, 0.25, np.float32)])[0]
    eng.index_add_records(7, recs)
    svc.register_tracks({"bulk-7": 7})
    assert svc.query(_pcm_of(0.25))[0].reference_path == "bulk-7"
    assert svc.index_track(_pcm_of(0.35), "next") and svc._ids["next"] == 8
    svc.checkpoint()
    again = fp.FingerprintService(tmp_path / "db")
    assert again.query(_pcm_of(0.25))[0].reference_path == "bulk-7"


def test_pipelined_service_batches_equal_serial(svc):
    """The service's coalescer runs its batches through the engine's submit / collect halves (pipelined dispatch):
    concurrent olaf_query calls get exactly the rows of serial queries; pipeline=False keeps the one-call path."""
    for i in range(4):
        assert run(fp.olaf_index_track(_pcm_of(0.1 * (i + 1)), uuid.UUID(int=4000 + i)))
    pcms = [_pcm_of(0.1 * (i % 5 + 1)) for i in range(24)]
    serial = [svc.query(p) for p in pcms]

    async def many():
        return await asyncio.gather(*[fp.olaf_query(p) for p in pcms])

    assert run(many()) == serial
    assert svc._eng().submits >= 1
    assert svc._coalescer._submit is not None
    off = fp.FingerprintService(svc.db_dir, pipeline=False)
    assert off._coalescer._submit is None
