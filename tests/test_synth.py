"""The synthetic generator (aidfp/synth.py), host side: generator v2's musical structure and its
rate independence, v0 kept for the golden fixture. (GPU == host bit for bit: tests/test_gpu_extract.py.)"""

import numpy as np

from aidfp import synth


def test_v2_tempo_and_onsets_per_track():
    lens = set()
    for tr in range(40):
        nl, offs = synth.note_params(tr, 44100)
        assert (44100 // 4) * 12 // 16 <= nl <= (44100 // 4) * 20 // 16  # 0.1875 .. 0.3125 s
        assert all(0 <= o < nl for o in offs) and len(set(offs)) > 1  # partials start at their own phases
        lens.add(nl)
    assert len(lens) >= 5  # tracks differ in tempo
    assert synth.note_params(3, 44100, envelope=False) == (44100 // 4, [0] * synth.N_PARTIALS)


def test_v2_notes_decay():
    """Every note decays linearly from full to half amplitude: the partials' mean power is E[(1 - u / 2)^2] = 7 / 12 of
    the stationary v0 notes' (same amplitude draws), within sampling error."""
    sr = 16000
    r = []
    for tr in range(6):
        v2 = synth.synth_int16(tr, 0, 20 * sr, sr).astype(np.float64)
        v0 = synth.synth_int16(tr, 0, 20 * sr, sr, envelope=False).astype(np.float64)
        r.append(np.mean(v2 ** 2) / np.mean(v0 ** 2))
    assert 0.45 < float(np.mean(r)) < 0.72, r


def test_same_music_at_every_rate():
    """v2's tempo and onsets are fractions of the note length, so a track's notes start at the same times (within a
    sample) at 16, 44.1 and 48 kHz: the capture at one rate and the catalog at another hold the same music."""
    for tr in (1, 2, 99):
        t = []
        for sr in (16000, 44100, 48000):
            nl, offs = synth.note_params(tr, sr)
            t.append((nl / sr, [o / sr for o in offs]))
        for nl_s, off_s in t[1:]:
            assert abs(nl_s - t[0][0]) < 2.0 / 16000
            assert max(abs(a - b) for a, b in zip(off_s, t[0][1])) < 2.0 / 16000


def test_v0_unchanged_by_v2():
    """envelope=False is the round-1..3 generator: its samples must not move (the golden fixture pins them too)."""
    x = synth.synth_int16(5, 123, 4000, 44100, envelope=False)
    assert x.dtype == np.int32 and len(x) == 4000
    i = np.arange(123, 4123, dtype=np.int64)
    j = i // (44100 // 4)
    # first partial's note index is the global 250 ms grid
    assert np.all(np.diff(j) >= 0) and j[0] == 0
    assert not np.array_equal(x, synth.synth_int16(5, 123, 4000, 44100))
