"""Batched exact lane (aid_exact_lane: GPU sub-window fan-out + K1-K5 + consensus kernel) against
the per-window path -- three olaf_query calls per <= 5 s clip merged by aidfp.exact's consensus,
which tests/test_glue_parity.py pins to vectors captured from the reference
(app/search/exact.py:70-353). Results must be identical: tracks, aligned counts, binary64
offsets and confidences, order."""

import asyncio
import uuid

import numpy as np
import pytest

from aidfp import exact as ex
from aidfp import fingerprint as fp
from aidfp import synth
from aidfp.engine import Engine

pytestmark = pytest.mark.gpu
SR = 16000
N_TRACKS = 24
IDS = [uuid.UUID(int=0xE000 + i) for i in range(N_TRACKS)]


def tr(track, start_s, n, snr=None, salt=0):
    return synth.synth(track, int(start_s * SR), int(n), SR, snr_db=snr, salt=salt)


@pytest.fixture(scope="module")
def service(tmp_path_factory):
    svc = fp.FingerprintService(tmp_path_factory.mktemp("exact_db"))
    svc.persist = False
    # a low engine min_match gives every window many rows, so the consensus sees multi-track,
    # single-window and halved candidates
    svc._engine = Engine(SR, device=0, min_match=4)
    for i, tid in enumerate(IDS):
        assert svc.index_track(tr(i, 0, 30 * SR).astype("<f4").tobytes(), str(tid))
    yield svc
    svc.close()


def clips():
    rng = np.random.default_rng(5)
    out = [np.zeros(0, np.float32), tr(1, 3.0, 800), tr(2, 1.0, SR), tr(3, 4.0, 2.2 * SR, snr=20),
           tr(4, 2.0, 3.5 * SR), tr(5, 9.0, 3.5 * SR + 1), tr(6, 0.0, 4 * SR, snr=15), tr(7, 5.0, 5 * SR - 1),
           tr(8, 6.0, 5 * SR, snr=20), tr(9, 7.0, 5 * SR + 1), tr(10, 2.0, 6 * SR, snr=20), tr(11, 11.0, 9.3 * SR + 3),
           tr(999, 0.0, 5 * SR, snr=20)]
    # splices: track A then track B inside one 5 s clip -> single-window candidates (halved)
    for a, b, cut in ((12, 13, 1.2), (14, 15, 2.6), (16, 17, 3.9)):
        x = tr(a, 8.0, 5 * SR, snr=25)
        x[int(cut * SR):] = tr(b, 3.0, 5 * SR - int(cut * SR), snr=25)
        out.append(x)
    # mixtures: two tracks at once -> two (or more) candidates per window, ties in confidence
    for a, b in ((18, 19), (20, 21), (22, 23)):
        out.append(np.clip(0.5 * tr(a, 4.0, 4.5 * SR) + 0.5 * tr(b, 10.0, 4.5 * SR), -1, 1).astype(np.float32))
    for k in range(6):  # random lengths and offsets
        t = int(rng.integers(0, N_TRACKS))
        out.append(tr(t, float(rng.uniform(0, 20)), int(rng.integers(SR // 2, 8 * SR)), snr=20, salt=k))
    return out


def _per_window(service, pcm, max_results):
    async def query(piece):
        return service.query(piece)

    return asyncio.run(ex.run_exact_lane(pcm, max_results, query=query))


@pytest.mark.parametrize("max_results", [3, 10, 50])
def test_batched_lane_equals_per_window_path(service, max_results):
    cs = [c.astype("<f4").tobytes() for c in clips()]
    got = asyncio.run(ex.run_exact_lane_batch(cs, max_results, service=service))
    assert len(got) == len(cs)
    nonempty = multi = 0
    for i, pcm in enumerate(cs):
        want = _per_window(service, pcm, max_results) if pcm else []
        assert got[i] == want, (i, got[i], want)
        nonempty += bool(want)
        multi += len(want) >= 2
    assert nonempty >= 12 and multi >= 3


def test_engine_rows_rank_order(service):
    """The raw kernel output: ranks by confidence (stable), aligned >= 8, confidence = min(h/20, 1)."""
    rows = service._engine.exact_lane(clips())
    for r in rows:
        if len(r) == 0:
            continue
        assert (r["aligned_hashes"] >= ex.MIN_ALIGNED_HASHES).all()
        assert np.array_equal(r["confidence"], np.minimum(r["aligned_hashes"] / 20.0, 1.0))
        assert (np.diff(r["confidence"]) <= 0).all()
        assert len(set(r["track"].tolist())) == len(r)


def test_device_pcm_and_many_clips(service):
    """Device PCM input and a batch larger than one K5 launch worth of windows."""
    import torch

    base = clips()[3:12]
    many = [base[i % len(base)] for i in range(700)]
    flat = np.concatenate(many)
    off = np.zeros(len(many) + 1, np.int64)
    off[1:] = np.cumsum([len(c) for c in many])
    dev = torch.from_numpy(flat).cuda()
    a = service._engine.exact_lane(pcm_ptr=dev.data_ptr(), offsets=off)
    b = service._engine.exact_lane(many)
    ref = service._engine.exact_lane(base)
    for i in range(len(many)):
        assert np.array_equal(a[i], b[i]) and np.array_equal(a[i], ref[i % len(base)])


def test_lane_rows_under_clip_groups(service):
    """The lane's windows split into several K1 -> K2 groups (engine.cpp extract_locked; `plane_rows` forces a
    small bound) give the same rows as one group."""
    base = clips()[3:12]
    many = [base[i % len(base)] for i in range(120)]
    eng = service._engine
    ref = eng.exact_lane(many)
    try:
        for rows in (300, 5000):
            eng.force("plane_rows", rows)
            got = eng.exact_lane(many)
            for i in range(len(many)):
                assert np.array_equal(got[i], ref[i]), f"plane_rows {rows}, clip {i}: rows differ"
    finally:
        eng.force("plane_rows", 0)


def test_single_clip_default_path(service):
    fp.set_service(service)
    try:
        res = asyncio.run(ex.run_exact_lane(tr(6, 12.0, 5 * SR, snr=20).astype("<f4").tobytes()))
    finally:
        fp.set_service(None)
    assert res and res[0].track == IDS[6] and res[0].confidence == 1.0
    assert abs(res[0].offset_seconds - 12.75) < 0.5


def test_lane_at_44k_odd_windows():
    """At 44.1 kHz the 0.75 s sub-window starts at an odd sample (33075) and windows can have odd
    lengths: the lane stages them even and extracts n - 1 samples of an odd window (same frames
    for an even hop). Rows must equal the per-window path on the engine's own queries."""
    sr = 44100
    eng = Engine(sr, device=0, min_match=5)
    try:
        tracks = np.arange(12, dtype=np.uint32) + 300
        for t in tracks:
            eng.index_add_records(int(t), eng.extract_host([synth.synth(int(t), 0, 20 * sr, sr)])[0])
        eng.index_finalize()
        cs = [synth.synth(int(tracks[i % 12]), sr * (i + 1) + 7 * i, n, sr, snr_db=20, salt=i)
              for i, n in enumerate([5 * sr, 5 * sr - 1, 4 * sr + 3, int(3.3 * sr) + 1, 2 * sr + 1, 6 * sr + 1,
                                     sr // 3, 5 * sr + 2])]
        names = {int(t): str(uuid.UUID(int=int(t))) for t in tracks}
        sec = eng.hop / eng.sample_rate

        async def query(piece):
            x = np.frombuffer(piece, dtype="<f4")
            eng.extract_host([x])
            rows = eng.query_extracted()[0]
            return [fp.OlafMatch(int(c), q0 * sec, q1 * sec, names[int(t)], int(t), (q0 + d) * sec, (q1 + d) * sec)
                    for c, t, d, q0, q1 in rows.tolist()]

        lane = eng.exact_lane(cs)
        eng.force("lane_gather", 1)  # the A/B: sub-windows copied to even offsets first
        try:
            staged = eng.exact_lane(cs)
        finally:
            eng.force("lane_gather", 0)
        assert all(np.array_equal(a, b) for a, b in zip(lane, staged))
        for i, x in enumerate(cs):
            want = asyncio.run(ex.run_exact_lane(x.astype("<f4").tobytes(), 10, query=query, sample_rate=sr))
            got = ex.candidates_from_rows(lane[i], names, 10)
            assert [(c.track_uuid, c.aligned_hashes, c.offset_seconds, c.confidence) for c in got] == \
                   [(m.track, m.aligned_hashes, m.offset_seconds, m.confidence) for m in want], i
    finally:
        eng.close()


def test_extract_device_odd_offsets():
    """Device clips at odd offsets (4-byte aligned float2 frame loads in K1) give the records of the
    same samples extracted from host copies."""
    import torch

    sr = 44100
    eng = Engine(sr, device=0)
    try:
        x = np.ascontiguousarray(synth.synth(7, 0, 3 * sr + 5, sr, snr_db=20, salt=3), dtype=np.float32)
        off = np.array([1, 33075, 66157, 66157 + sr + 2, 3 * sr + 5], np.int64)
        dev = torch.from_numpy(x).cuda()
        eng.extract_device(dev.data_ptr(), off)
        eng.sync()
        got = [eng.hashes(c) for c in range(len(off) - 1)]
        want = eng.extract_host([x[off[c]:off[c + 1]] for c in range(len(off) - 1)])
        for c in range(len(off) - 1):
            assert len(want[c]) > 0 or off[c + 1] - off[c] < sr // 4
            assert np.array_equal(got[c], want[c]), c
    finally:
        eng.close()
