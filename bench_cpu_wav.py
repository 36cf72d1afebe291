#!/usr/bin/env python3
"""BASELINE config 1: one 10 s 44.1 kHz mono WAV through the CPU fingerprint path (plumbing, no GPU).

SURVEY.md 8d config 1: the reference's own path would be ffmpeg decode -> olaf_c (external,
absent here); the CPU path of this repo is the bit-exact C restatement of FPSPEC
(oracle/fp_oracle.c -- test infrastructure and CPU baseline, never the product path). The clip
is a synthetic int16 WAV written and read back with scipy.io.wavfile (ffmpeg is not in the
image), converted to f32 as ffmpeg's f32le output would be (sample / 32768, exact).

    python bench_cpu_wav.py [--seconds 10] [--repeat 20] [--gpu]

--gpu also fingerprints the decoded clip on the MI355X and checks the hashes are identical.
"""

from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path[:0] = [str(ROOT / "audio-ident_amd"), str(ROOT / "oracle")]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--sr", type=int, default=44100)
    ap.add_argument("--repeat", type=int, default=20)
    ap.add_argument("--gpu", action="store_true")
    args = ap.parse_args()

    from scipy.io import wavfile

    import oracle as O  # the CPU path (checker / baseline)
    from aidfp import synth

    n = int(args.seconds * args.sr)
    q = synth.synth_int16(42, 0, n, args.sr, synth.noise_halfwidth(30.0)).astype(np.int16)
    with tempfile.TemporaryDirectory() as d:
        path = Path(d) / "clip.wav"
        wavfile.write(path, args.sr, q)
        t0 = time.perf_counter()
        sr, data = wavfile.read(path)
        x = (data.astype(np.float32) / np.float32(32768.0)).astype(np.float32)
        t_decode = time.perf_counter() - t0
    hop = O.default_hop(sr)
    O.fingerprint(x[: 2 * 2048], hop)  # warm (tables, library load)
    t0 = time.perf_counter()
    for _ in range(args.repeat):
        recs = O.fingerprint(x, hop)
    t_fp = (time.perf_counter() - t0) / args.repeat
    out = {
        "metric": "CPU plumbing: 10 s 44.1 kHz mono WAV -> landmark hashes (oracle/fp_oracle.c, 1 thread)",
        "value": round(args.seconds / t_fp, 1), "unit": "audio-s/s", "seconds": args.seconds, "sample_rate": sr,
        "wav_read_ms": round(t_decode * 1e3, 3), "fingerprint_ms": round(t_fp * 1e3, 3), "hashes": int(len(recs)),
        "frames": O.num_frames(len(x), hop), "cores": 1, "data": "synthetic int16 WAV (aid_synth track 42, -30 dB noise)",
    }
    if args.gpu:
        from aidfp.engine import Engine

        with Engine(sr) as eng:
            got = eng.extract_host([x])[0]
        out["gpu_hashes_identical"] = bool(np.array_equal(got, recs))
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
