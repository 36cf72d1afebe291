"""Pins the CPU oracle (oracle/fp_oracle.c) -- the checker every GPU parity test
trusts. The reference holds no golden vectors for this arithmetic (it lives in
the external olaf_c binary, SURVEY.md 8c: parity unpinned by the reference), so
the oracle is pinned here by:
  * float64 numpy rfft power (tolerance);
  * the literal FPSPEC 5 peak definition (brute force) vs the separable form;
  * known-answer cases (bin-centred sinusoids, hand-built peak lists);
  * the committed golden fixtures tests/golden/oracle_v0.npz (extraction) and oracle_match_v1.npz (FPSPEC v1
    match: distinct anchor frames), as regression locks.
"""

import json
from pathlib import Path

import numpy as np
import pytest

import oracle as O
from aidfp import synth

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_num_frames():
    assert O.num_frames(0, 512) == 0
    assert O.num_frames(2047, 512) == 0
    assert O.num_frames(2048, 512) == 1
    assert O.num_frames(2048 + 511, 512) == 1
    assert O.num_frames(2048 + 512, 512) == 2
    assert O.num_frames(441000, 512) == 858


@pytest.mark.parametrize("tr,snr", [(1, None), (2, 20.0), (3, 5.0)])
def test_power_matches_float64(tr, snr):
    x = synth.synth(tr, 999, 60000, 44100, snr_db=snr, salt=3)
    P = O.stft_power(x, 512).astype(np.float64)
    P64 = O.stft_power_f64(x, 512)
    # binary32 FFT error relative to each frame's peak power
    assert (np.abs(P - P64) / P64.max(axis=1, keepdims=True)).max() < 2e-6


def test_bin_centred_sine_peak():
    # a sine exactly on bin 100 of a 2048-point frame peaks at bin 100 in every frame
    n = 2048 + 512 * 40
    t = np.arange(n)
    x = (0.25 * np.sin(2 * np.pi * 100 * t / 2048)).astype(np.float32)
    P = O.stft_power(x, 512)
    assert (P.argmax(axis=1) == 100).all()
    # |X[100]|^2 = (A * N/4)^2 for a periodic Hann window (sum w = N/2)
    assert np.allclose(P[:, 100], (0.25 * 2048 / 4) ** 2, rtol=1e-4)
    pk = O.peaks(P)
    assert len(pk) >= 1 and (pk[:, 1] == 100).all()


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_separable_peaks_equal_bruteforce(seed):
    rng = np.random.default_rng(seed)
    x = synth.synth(10 + seed, 0, 2048 + 512 * 60, 44100, snr_db=10.0, salt=seed)
    P = O.stft_power(x, 512)
    assert np.array_equal(O.peaks(P), O.peaks(P, brute=True))
    # plateaus and exact ties: quantised random powers force equal values in a neighbourhood
    Q = np.round(rng.random((50, 1024)) * 8).astype(np.float32) * 4.0
    assert np.array_equal(O.peaks(Q), O.peaks(Q, brute=True))
    # flat field: every point has an earlier tied neighbour (bin 0 / row above), so no peaks
    Z = np.full((20, 1024), 7.0, np.float32)
    assert len(O.peaks(Z)) == 0 and len(O.peaks(Z, brute=True)) == 0


def test_peak_packing_bound():
    rng = np.random.default_rng(5)
    for F in (1, 7, 8, 9, 64):
        Q = (rng.random((F, 1024)) * 100 + 5).astype(np.float32)
        n = len(O.peaks(Q))
        assert n <= 64 * ((F + 7) // 8)


def test_hash_known_answer():
    pk = np.array([[0, 100], [1, 90], [1, 300], [5, 227], [64, 100], [70, 101]], dtype=np.int32)
    rec = O.hashes_from_peaks(pk)
    h = (rec & np.uint64(0xFFFFFFFF)).astype(np.int64)
    t1 = (rec >> np.uint64(32)).astype(np.int64)

    def H(k1, k2, dt):
        return (k1 << 22) | (k2 << 12) | dt

    # anchor (0,100): (1,90) ok, (1,300) |df|=200 > 127 skip, (5,227) df=127 ok, (64,100) dt=64 > 63 stop
    # anchor (1,90): (1,300) dt=0 skip, (5,227) df=137 skip, (64,100) dt=63 ok, (70,101) dt=69 stop
    # anchor (1,300): (5,227) ok, (64,100) df=-200 skip; (5,227): (64,100) df=-127 ok; (64,100): (70,101)
    expect = [(H(100, 90, 1), 0), (H(100, 227, 5), 0), (H(90, 100, 63), 1), (H(300, 227, 4), 1),
              (H(227, 100, 59), 5), (H(100, 101, 6), 64)]
    assert list(zip(h.tolist(), t1.tolist())) == expect


def test_fanout_limit():
    pk = np.array([[0, 500]] + [[1 + i, 500 + i] for i in range(15)], dtype=np.int32)
    rec = O.hashes_from_peaks(pk)
    t1 = (rec >> np.uint64(32)).astype(np.int64)
    assert (t1 == 0).sum() == 10


def test_fingerprint_equals_staged_pipeline():
    x = synth.synth(4, 0, 100000, 44100)
    staged = O.hashes_from_peaks(O.peaks(O.stft_power(x, 512)))
    assert np.array_equal(O.fingerprint(x, 512), staged)
    b = O.fingerprint_batch(np.stack([x, x]), 512, threads=2)
    assert np.array_equal(b[0], staged) and np.array_equal(b[1], staged)


def test_golden_fixture_regression():
    """Oracle outputs on committed inputs must not drift (tests/golden/make_oracle_golden.py)."""
    g = np.load(GOLDEN / "oracle_v0.npz")
    meta = json.loads((GOLDEN / "oracle_v0.json").read_text())
    for i, spec in enumerate(meta["clips"]):
        # the fixture was made with the v0 generator (stationary notes)
        x = synth.synth(spec["track"], spec["start"], spec["n"], spec["sr"], snr_db=spec["snr"], salt=spec["salt"],
                        envelope=spec.get("envelope", False))
        assert np.array_equal(x, g[f"pcm_{i}"]), "synth drifted"
        assert np.array_equal(O.fingerprint(x, spec["hop"]), g[f"rec_{i}"]), f"clip {i} hashes drifted"
        P = O.stft_power(x, spec["hop"])
        assert np.array_equal(P[:4], g[f"pow_{i}"]), f"clip {i} power drifted"


def test_match_oracle_votes():
    # track 7 holds hashes at t = 100.., query holds the same hashes at t = 0.. -> d = 100
    post = np.array([[11, 7, 100], [12, 7, 101], [13, 7, 102], [11, 8, 5], [99, 9, 1]], dtype=np.uint32)
    q = np.array([11, 12, 13, 11], dtype=np.uint64) | (np.array([0, 1, 2, 50], dtype=np.uint64) << np.uint64(32))
    rows = O.query(post, q, min_match=1)
    assert rows[0].tolist() == [3, 7, 100, 0, 2]
    assert sorted(r[1] for r in rows) == [7, 8]


def test_match_oracle_counts_distinct_anchor_frames():
    """FPSPEC v1 7: a (track, d) scores the DISTINCT query anchor frames among its votes. Query frame 0 holds two
    records (hashes 11 and 14) that both vote (7, d = 100): 4 votes, 3 distinct frames -> match_count 3. Track 8
    gets 3 votes for d = 40, all from frame 10 (one onset's harmonics): match_count 1, below min_match 2."""
    post = np.array([[11, 7, 100], [14, 7, 100], [12, 7, 101], [13, 7, 102],
                     [21, 8, 50], [22, 8, 50], [23, 8, 50]], dtype=np.uint32)
    qh = np.array([11, 14, 12, 13, 21, 22, 23], dtype=np.uint64)
    qt = np.array([0, 0, 1, 2, 10, 10, 10], dtype=np.uint64)
    rows = O.query(post, qh | (qt << np.uint64(32)), min_match=1)
    assert rows.tolist() == [[3, 7, 100, 0, 2], [1, 8, 40, 10, 10]]
    rows = O.query(post, qh | (qt << np.uint64(32)), min_match=2)
    assert rows.tolist() == [[3, 7, 100, 0, 2]]


def test_numpy_scipy_path_matches_on_synthetic_clips():
    """The bench's NumPy/SciPy cpu_baseline leg (float64 FFT) gives the spec's records on the synthetic
    workloads (band-limited and full-band, clean and noisy): its timing is for the same output."""
    from aidfp import synth

    for tr, snr, fmax in ((3, None, 8000), (4, 20.0, 8000), (5, None, 20000)):
        x = synth.synth(tr, 0, 44100 * 4, 44100, snr_db=snr, fmax_hz=fmax)
        assert np.array_equal(O.fingerprint_numpy(x, 512), O.fingerprint(x, 512))


def test_match_v1_golden_fixture():
    """FPSPEC v1 section 7 regression vectors (tests/golden/make_match_golden.py): the oracle's rows from the committed
    postings and query records at min_match 10 and 4; every v1 score is at most the v0 vote count of its (track, d),
    and the two differ (what v1 changed)."""
    g = np.load(GOLDEN / "oracle_match_v1.npz")
    meta = json.loads((GOLDEN / "oracle_match_v1.json").read_text())
    post = g["postings"]
    differ = 0
    for i in range(len(meta["queries"])):
        rec = g[f"rec_{i}"]
        for mm in (10, 4):
            assert np.array_equal(O.query(post, rec, min_match=mm, max_rows=50), g[f"rows_mm{mm}_{i}"]), (i, mm)
        rows, v0 = g[f"rows_mm4_{i}"], g[f"v0votes_{i}"]
        assert (rows[:, 0] <= v0).all() if len(rows) else True
        differ += int((rows[:, 0] < v0).sum()) if len(rows) else 0
    assert differ > 0
