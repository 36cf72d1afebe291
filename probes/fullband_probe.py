"""K2 strip sizing on band-limited vs full-band audio: the bench batch (partials <= 8 kHz, -40 dBFS noise)
and the same batch with uniform noise loud enough that most 64-bin blocks are hot at every frequency.
Prints the per-launch K1/K2/K3 times for the engine's adaptive sizing (AIDFP_K2_SLOTS_X unset) or the
fixed multiplier given in the environment. Diagnostic only.

usage: [AIDFP_K2_SLOTS_X=1.5] python probes/fullband_probe.py
"""
import json
import os
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
    return {"ms_per_step": round(dt * 1e3, 4),
            **{k: round(ms / n, 4) for k, (ms, n) in prof.items() if n}}


def main():
    import torch

    from aidfp.engine import Engine

    eng = Engine(44100, device=0)
    n = 441000
    clips = 256
    pcm = torch.empty(clips * n, dtype=torch.float32, device="cuda")
    offs = np.arange(clips + 1, dtype=np.int64) * n
    tracks = np.arange(clips, dtype=np.uint32)
    out = {"slots_x": os.environ.get("AIDFP_K2_SLOTS_X", "adaptive")}
    eng.synth(pcm.data_ptr(), tracks, np.zeros(clips, np.int64), n)
    out["band_limited"] = run(eng, pcm, offs)
    eng.synth(pcm.data_ptr(), tracks, np.zeros(clips, np.int64), n, noise_a=6000)  # ~-15 dBFS uniform noise
    out["full_band"] = run(eng, pcm, offs)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
