"""The drop-in API end to end on the GPU (16 kHz, the reference's boundary rate):
olaf_index_track / olaf_query / olaf_delete_track through libaidfp.so, and the
exact lane (sub-window consensus for <= 5 s clips, full clip otherwise)
identifying the right track and offset. Mirrors what the reference's
scripts/eval_exact.py measures (top-1 track, offset error < 0.5 s)."""

import asyncio
import uuid

import numpy as np
import pytest

from aidfp import exact as ex
from aidfp import fingerprint as fp
from aidfp import synth

pytestmark = pytest.mark.gpu
SR = 16000
IDS = [uuid.UUID(int=0xA000 + i) for i in range(6)]


def pcm_bytes(track, start_s, dur_s, snr=None, salt=0):
    x = synth.synth(track, int(start_s * SR), int(dur_s * SR), SR, snr_db=snr, salt=salt)
    return x.astype("<f4").tobytes()


@pytest.fixture(scope="module")
def service(tmp_path_factory):
    db = tmp_path_factory.mktemp("olaf_db")
    svc = fp.FingerprintService(db)
    fp.set_service(svc)
    for i, tid in enumerate(IDS):
        assert asyncio.run(fp.olaf_index_track(pcm_bytes(i, 0, 30), tid))
    yield svc, db
    fp.set_service(None)
    svc.close()


def test_query_identifies_track(service):
    res = asyncio.run(fp.olaf_query(pcm_bytes(3, 7.0, 5.0, snr=20, salt=1)))
    assert res and res[0].reference_path == str(IDS[3])
    assert res[0].reference_start == pytest.approx(7.0 + res[0].query_start, abs=0.05)


@pytest.mark.parametrize("dur,start", [(5.0, 7.0), (4.0, 12.0), (8.0, 3.0)])
def test_exact_lane(service, dur, start):
    res = asyncio.run(ex.run_exact_lane(pcm_bytes(2, start, dur, snr=20, salt=2)))
    assert res and res[0].track == IDS[2] and res[0].confidence == 1.0
    # reference quirk (exact.py:263-270): the offset is the median raw reference_start,
    # i.e. start + the window's position in the clip for sub-windowed queries
    expect = start + (0.75 if dur <= 5.0 else 0.0)
    assert abs(res[0].offset_seconds - expect) < 0.5


def test_unknown_audio_no_match(service):
    assert asyncio.run(ex.run_exact_lane(pcm_bytes(999, 0, 5.0, snr=20))) == []


def test_delete_and_reload(service):
    svc, db = service
    assert asyncio.run(fp.olaf_delete_track(IDS[5]))
    assert not asyncio.run(fp.olaf_delete_track(IDS[5]))
    res = asyncio.run(fp.olaf_query(pcm_bytes(5, 10.0, 6.0)))
    assert all(m.reference_path != str(IDS[5]) for m in res)
    # a new service instance (process restart) reads the persisted index
    other = fp.FingerprintService(db)
    try:
        r = other.query(pcm_bytes(1, 4.0, 6.0))
        assert r and r[0].reference_path == str(IDS[1])
        assert all(m.reference_path != str(IDS[5]) for m in other.query(pcm_bytes(5, 10.0, 6.0)))
    finally:
        other.close()


def test_short_clip_store_delete_restore(tmp_path):
    """a clip shorter than one frame (2048 samples) gives no hashes; it is still
    stored, deletable and re-storable through the real engine, and survives a restart."""
    svc = fp.FingerprintService(tmp_path / "db")
    tid = uuid.UUID(int=0xBEEF)
    short = np.full(1500, 0.1, dtype="<f4").tobytes()
    try:
        assert svc.index_track(short, str(tid))
        assert svc.delete_track(str(tid))
        assert svc.index_track(short, str(tid))
        assert svc.index_track(short, str(tid))  # re-store over a zero-hash track
        assert svc.index_track(pcm_bytes(4, 0, 20), "full")
        svc.checkpoint()  # snapshot + compaction of the replaced ids
    finally:
        svc.close()
    again = fp.FingerprintService(tmp_path / "db")
    try:
        assert again.delete_track(str(tid))
        r = again.query(pcm_bytes(4, 6.0, 6.0))
        assert r and r[0].reference_path == "full"
    finally:
        again.close()
