"""K2 strip sizing on band-limited vs full-band audio: the bench batch (partials <= 8 kHz) and the bench's full-band
batch (partials <= 20 kHz), extracted with the engine's adaptive strip sizing and with fixed strips-per-slot
multipliers (aid_engine_force K2_STRIPS_X100). Prints per-launch K1/K2/K3 times per setting. Diagnostic only.

usage: python probes/fullband_probe.py [x100 ...]     (0 = adaptive; default: 0 100 125 150 175 200)
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "audio-ident_amd"))


def run(eng, pcm, offs, steps=40):
    import torch

    for _ in range(60):  # warm up + let the adaptive sizing see a few counts
        eng.extract_device(pcm.data_ptr(), offs)
    torch.cuda.synchronize()
    eng.profile_select(None)
    eng.profile_enable(True)
    eng.profile_read(reset=True)
    t = time.perf_counter()
    for _ in range(steps):
        eng.extract_device(pcm.data_ptr(), offs)
    eng.sync()
    dt = (time.perf_counter() - t) / steps
    prof = eng.profile_read(reset=True)
    eng.profile_enable(False)
    return {"ms_per_step": round(dt * 1e3, 4), **{k: round(ms / n, 4) for k, (ms, n) in prof.items() if n}}


def main():
    import torch

    from aidfp.engine import Engine

    settings = [int(a) for a in sys.argv[1:]] or [0, 100, 125, 150, 175, 200]
    eng = Engine(44100, device=0)
    n, clips = 441000, 256
    pcm = torch.empty(clips * n, dtype=torch.float32, device="cuda")
    offs = np.arange(clips + 1, dtype=np.int64) * n
    tracks = np.arange(clips, dtype=np.uint32)
    out = {}
    for name, fmax in (("band_limited", 8000), ("full_band", 20000)):
        eng.synth(pcm.data_ptr(), tracks + (0 if fmax == 8000 else 500000), np.zeros(clips, np.int64), n, fmax_hz=fmax)
        for x in settings:
            eng.force("k2_strips_x100", x)
            out[f"{name}/{x or 'adaptive'}"] = run(eng, pcm, offs)
    eng.force("k2_strips_x100", 0)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
