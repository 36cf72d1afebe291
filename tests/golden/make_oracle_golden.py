"""Writes tests/golden/oracle_v0.{npz,json}: small regression vectors of the CPU
oracle (spec/FPSPEC.md v0) -- inputs (synthetic PCM) and outputs (first power
rows, landmark records). Run from the repo root: python tests/golden/make_oracle_golden.py
These lock the oracle against drift; they are NOT reference (olaf_c) outputs,
which do not exist offline (parity unpinned by the reference)."""

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "audio-ident_amd")]
import oracle as O  # noqa: E402
from aidfp import synth  # noqa: E402

CLIPS = [
    {"track": 1, "start": 0, "n": 44100 * 3, "sr": 44100, "hop": 512, "snr": None, "salt": 0},
    {"track": 2, "start": 12345, "n": 44100 * 2 + 77, "sr": 44100, "hop": 512, "snr": 20.0, "salt": 9},
    {"track": 3, "start": 0, "n": 16000 * 4, "sr": 16000, "hop": 256, "snr": None, "salt": 0},
    {"track": 4, "start": 500, "n": 48000 * 2, "sr": 48000, "hop": 512, "snr": 10.0, "salt": 1},
]

out = {}
for i, c in enumerate(CLIPS):
    x = synth.synth(c["track"], c["start"], c["n"], c["sr"], snr_db=c["snr"], salt=c["salt"],
                    envelope=c.get("envelope", False))  # oracle_v0.* holds v0-generator inputs
    out[f"pcm_{i}"] = x
    out[f"rec_{i}"] = O.fingerprint(x, c["hop"])
    out[f"pow_{i}"] = O.stft_power(x, c["hop"])[:4]
here = Path(__file__).resolve().parent
np.savez_compressed(here / "oracle_v0.npz", **out)
(here / "oracle_v0.json").write_text(json.dumps({"spec": "FPSPEC v0", "clips": CLIPS}, indent=1))
print({k: v.shape for k, v in out.items()})
