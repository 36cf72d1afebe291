"""Error contract and persistence of the drop-in aidfp.fingerprint module, in the
style of the reference's tests/test_audio_fingerprint.py (which mocks the olaf_c
subprocess): here the GPU engine class is replaced by a small test double so the
host logic runs without a GPU. The real engine path is covered by
tests/test_gpu_adapter.py."""

import asyncio
import uuid

import numpy as np
import pytest

from aidfp import _lib
from aidfp import cli
from aidfp import fingerprint as fp

TID = uuid.UUID("12345678-1234-5678-1234-567812345678")
PCM = np.arange(4000, dtype="<f4").tobytes()


class FakeEngine:
    """Test double of aidfp.engine.Engine: 'fingerprints' are the first PCM values."""

    def __init__(self, sample_rate, device=-1, fail=None):
        self.sample_rate, self.hop = sample_rate, 256
        self.tracks, self.removed, self.fail = {}, set(), fail
        self._last = None

    def extract_host(self, clips):
        if self.fail == "extract":
            raise _lib.EngineError(-1, "bad input")
        self._last = [np.asarray(c[:3], dtype=np.float32) for c in clips]
        return [np.arange(3, dtype=np.uint64) for _ in clips]

    def index_add_records(self, track, recs):
        self.tracks[track] = self._last[0]

    def index_remove(self, track):
        if track in self.removed or track not in self.tracks:
            raise _lib.EngineError(-1, "track not indexed")
        self.removed.add(track)

    def query_extracted(self):
        q = self._last[0]
        rows = [[10 + t, t, 4, 1, 20] for t, v in self.tracks.items() if t not in self.removed and np.array_equal(v, q)]
        rows += [[5, t, 0, 0, 2] for t in self.tracks if t not in self.removed and len(rows) < 3]
        return [np.array(rows, dtype=np.int64).reshape(-1, 5)]

    def index_save(self, path):
        open(path, "w").write("x")

    def index_load(self, path):
        pass

    def close(self):
        pass


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
    assert (tmp_path / "db" / "index.aidfp").exists() and (tmp_path / "db" / "tracks.json").exists()


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
