"""aid_exact_windows (host-only C ABI, no GPU) reproduces the reference's sub-window slicing:
app/search/exact.py duration (:389-390), SUB_WINDOWS (:48-52), stop = min(b, duration) and
`piece if a < stop else b""` (:150-160), _extract_pcm_window's int(t * SAMPLE_RATE) byte bounds
(:374-399) -- mirrored by aidfp.exact, whose outputs tests/test_glue_parity.py pins to the
reference. Checked for every length near the window edges at 16, 44.1 and 48 kHz."""

import pytest

from aidfp import exact as ex
from aidfp.engine import exact_windows


def _python_plan(n, sr):
    pcm = bytes(range(256)) * ((4 * n) // 256 + 1)
    pcm = pcm[: 4 * n]
    dur = ex.pcm_duration_sec(pcm, sr)
    if dur > ex.SHORT_CLIP_THRESHOLD_SEC:
        return 0, [(0, n)]
    out = []
    for a, b in ex.SUB_WINDOWS:
        stop = min(b, dur)
        if not a < stop:
            out.append((0, 0))
            continue
        lo = min(max(int(a * sr) * 4, 0), len(pcm))
        hi = max(lo, min(int(stop * sr) * 4, len(pcm)))
        piece = ex.extract_pcm_window(pcm, a, stop, sr)
        assert piece == pcm[lo:hi]
        out.append((lo // 4, (hi - lo) // 4) if hi > lo else (0, 0))
    return 1, out


@pytest.mark.parametrize("sr", [16000, 44100, 48000])
def test_windows_match_reference_slicing(sr):
    edges = [0, 1, 2, 2047, 2048, 2049]
    for t in (0.75, 1.5, 3.5, 4.25, 5.0):
        c = int(t * sr)
        edges += list(range(c - 3, c + 4))
    edges += [sr * 7 + 5, sr * 30]
    for n in sorted(set(e for e in edges if e >= 0)):
        mode, wins = exact_windows(n, sr)
        want_mode, want = _python_plan(n, sr)
        assert mode == want_mode, n
        got = [(lo, ln) if ln > 0 else (0, 0) for lo, ln in wins]
        assert got == want, (n, got, want)
