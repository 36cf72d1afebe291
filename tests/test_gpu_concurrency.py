"""Concurrent readers through the real engine: 64 olaf_query
requests in flight at once are coalesced into a few aid_query_pcm batches and return exactly the
rows a serial loop returns; a store and a delete interleaved with the queries neither corrupt nor
block them (RW lock: writers exclusive, readers shared). The reference runs one `olaf_c query`
subprocess per request (audio-ident-service/app/audio/fingerprint.py:185-193)."""

import asyncio
import threading
import uuid

import pytest

from aidfp import fingerprint as fp
from aidfp import synth

pytestmark = pytest.mark.gpu
SR = 16000
N_TRACKS = 24
IDS = [uuid.UUID(int=0xC000 + i) for i in range(N_TRACKS)]


def pcm_bytes(track, start_s, dur_s, snr=None, salt=0):
    x = synth.synth(track, int(start_s * SR), int(dur_s * SR), SR, snr_db=snr, salt=salt)
    return x.astype("<f4").tobytes()


def _queries(n):
    # a mix of known tracks at different offsets / lengths / noise and a few unknown clips
    qs = []
    for i in range(n):
        t = i % N_TRACKS if i % 8 else 1000 + i
        qs.append(pcm_bytes(t, 1.0 + (i * 0.37) % 20.0, 3.0 + (i % 5), snr=20 if i % 3 else None, salt=i))
    return qs


@pytest.fixture(scope="module")
def service(tmp_path_factory):
    svc = fp.FingerprintService(tmp_path_factory.mktemp("olaf_db_conc"), coalesce_window_s=0.002)
    fp.set_service(svc)
    for i, tid in enumerate(IDS):
        assert svc.index_track(pcm_bytes(i, 0, 30), str(tid))
    yield svc
    fp.set_service(None)
    svc.close()


def test_64_concurrent_queries_equal_serial(service):
    qs = _queries(64)
    serial = [service.query(q) for q in qs]
    assert sum(1 for r in serial if r) >= 50  # the known-track queries match
    service._coalescer.batches.clear()

    async def fan_out():
        return await asyncio.gather(*(fp.olaf_query(q) for q in qs))

    conc = asyncio.run(fan_out())
    assert conc == serial
    assert sum(service._coalescer.batches) == 64 and len(service._coalescer.batches) < 64  # coalesced


def test_queries_with_interleaved_writer(service):
    qs = _queries(48)
    serial = [service.query(q) for q in qs]
    extra = str(uuid.UUID(int=0xCFFF))
    errors = []

    def writer():
        try:
            for _ in range(3):
                assert service.index_track(pcm_bytes(5000, 0, 10), extra)
                assert service.delete_track(extra)
        except BaseException as exc:  # noqa: BLE001 -- surfaced below
            errors.append(exc)

    async def fan_out():
        return await asyncio.gather(*(fp.olaf_query(q) for q in qs))

    t = threading.Thread(target=writer)
    t.start()
    conc = asyncio.run(fan_out())
    t.join(timeout=60)
    assert not t.is_alive() and not errors
    # track 5000's audio is not among the queries, so its brief presence changes no row
    assert conc == serial


def test_query_pcm_submit_equals_query_pcm(service):
    """aid_query_pcm_submit (the coalescer's pipelined half): two batches in flight at once, each with its own
    page-locked PCM, collected out of order, give aid_query_pcm's rows bit for bit."""
    import numpy as np

    eng = service._eng()
    qs = [np.frombuffer(q, dtype="<f4") for q in _queries(24)]
    ref = eng.query_pcm(qs)
    a = eng.query_pcm_submit(qs[:12])
    b = eng.query_pcm_submit(qs[12:])
    got = b.collect()
    got = a.collect() + got
    assert len(got) == 24 and all(np.array_equal(x, y) for x, y in zip(got, ref))
    assert sum(len(r) > 0 for r in ref) >= 15
    assert eng.query_pcm_submit([]).collect() == []


def test_pipelined_batches_overlap_and_equal_serial(service):
    """Small batches (max_batch 8) under 64 requests in flight: the dispatcher starts batch N + 1 before it collects
    batch N, and every request still gets its serial rows."""
    qs = _queries(64)
    serial = [service.query(q) for q in qs]
    c = service._coalescer
    keep = c.max_batch
    c.max_batch = 8
    c.overlapped = 0
    try:
        async def fan_out():
            return await asyncio.gather(*(fp.olaf_query(q) for q in qs))

        assert asyncio.run(fan_out()) == serial
        assert c.overlapped > 0
    finally:
        c.max_batch = keep
