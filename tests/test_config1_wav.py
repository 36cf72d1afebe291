"""BASELINE config 1 (CPU plumbing, no GPU): a 10 s 44.1 kHz mono int16 WAV, written and read back
with scipy.io.wavfile (ffmpeg is not in the image), decoded to f32 as ffmpeg's f32le (x / 32768,
exact), fingerprinted by the CPU path (oracle/fp_oracle.c) -- the same records as fingerprinting
the synthetic samples directly, and the bench script's JSON line is well formed."""

import json
import subprocess
import sys
from pathlib import Path

import numpy as np

import oracle as O
from aidfp import synth

ROOT = Path(__file__).resolve().parents[1]


def test_wav_roundtrip_is_exact_and_fingerprints(tmp_path):
    from scipy.io import wavfile

    sr, n = 44100, 441000
    q = synth.synth_int16(42, 0, n, sr, synth.noise_halfwidth(30.0)).astype(np.int16)
    wavfile.write(tmp_path / "clip.wav", sr, q)
    sr2, data = wavfile.read(tmp_path / "clip.wav")
    assert sr2 == sr and data.dtype == np.int16 and len(data) == n
    x = (data.astype(np.float32) / np.float32(32768.0)).astype(np.float32)
    direct = synth.synth(42, 0, n, sr, snr_db=30.0)
    assert np.array_equal(x, direct)
    recs = O.fingerprint(x, O.default_hop(sr))
    assert 1000 < len(recs) and np.array_equal(recs, O.fingerprint(direct, O.default_hop(sr)))


def test_bench_cpu_wav_line():
    out = subprocess.run([sys.executable, str(ROOT / "bench_cpu_wav.py"), "--repeat", "2"], capture_output=True,
                         text=True, timeout=300, check=True)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["unit"] == "audio-s/s" and d["value"] > 0 and d["hashes"] > 1000 and d["frames"] == 858
