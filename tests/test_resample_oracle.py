"""The PCM front-end oracle (oracle/fp_resample.c, FPSPEC 8) pinned to the published algorithm it
restates: scipy.signal.resample_poly (scipy 1.15.3, Kaiser beta 5). The reference's own front-end
is ffmpeg (`decode.py:41-60`), which is absent here, so scipy is the anchor ("parity pinned to
scipy", not to ffmpeg)."""

import numpy as np
import pytest
import scipy.signal as ss

import oracle as O

RATES = [(48000, 16000), (48000, 44100), (44100, 16000), (16000, 48000), (44100, 48000), (22050, 16000),
         (96000, 44100), (8000, 44100)]


@pytest.mark.parametrize("sr_in,sr_out", RATES)
def test_taps_equal_scipy_firwin(sr_in, sr_out):
    up, down, hl, J = O.resample_ratio(sr_in, sr_out)
    h = ss.firwin(2 * hl + 1, 1.0 / max(up, down), window=("kaiser", 5.0)) * up
    t = O.resample_taps(sr_in, sr_out)
    assert t.shape == h.shape
    # binary64 design rounded once: equal to scipy's taps rounded to binary32 (1 ulp slack for
    # the different summation order of the DC normalisation)
    ulps = np.abs(t.view(np.int32).astype(np.int64) - h.astype(np.float32).view(np.int32).astype(np.int64))
    assert ulps.max() <= 1


@pytest.mark.parametrize("sr_in,sr_out", RATES)
def test_output_matches_scipy_resample_poly(sr_in, sr_out):
    rng = np.random.default_rng(sr_in + sr_out)
    x = (rng.standard_normal(sr_in // 3 + 17) * 0.3).astype(np.float32)
    up, down, _, _ = O.resample_ratio(sr_in, sr_out)
    y = O.resample(x, sr_in, sr_out)
    yr = ss.resample_poly(x.astype(np.float64), up, down)
    assert len(y) == len(yr)
    assert np.max(np.abs(y - yr)) <= 2e-6 * (1 + np.max(np.abs(x)))


def test_stereo_downmix_then_resample():
    rng = np.random.default_rng(3)
    st = (rng.standard_normal((48000, 2)) * 0.4).astype(np.float32)
    mono = ((st[:, 0] + st[:, 1]) * np.float32(0.5)).astype(np.float32)
    assert np.array_equal(O.resample(st, 48000, 16000), O.resample(mono, 48000, 16000))


def test_edges():
    x = np.ones(5, np.float32)
    assert len(O.resample(np.zeros(0, np.float32), 48000, 16000)) == 0
    y = O.resample(x, 48000, 16000)  # shorter than the filter
    assert len(y) == 2
    assert np.array_equal(O.resample(x, 16000, 16000), x)  # same rate: copy
    # a pure in-band tone keeps its amplitude (gain 1 at DC)
    t = np.arange(48000) / 48000.0
    tone = (0.5 * np.sin(2 * np.pi * 440.0 * t)).astype(np.float32)
    y = O.resample(tone, 48000, 16000)
    assert abs(np.max(np.abs(y[2000:-2000])) - 0.5) < 1e-3
