"""VERDICT r5 next #3, second half: does K2's load latency shrink when a K1 -> K2 group's power plane fits the 256 MiB
Infinity Cache (MALL)? The headline batch (256 x 10 s at 44.1 kHz, band-limited and full-band) is extracted with the
engine's clip groups forced to N clips' rows (aid_engine_force PLANE_ROWS: 858 rows per clip, 3.5 MB each; 64 clips
= 225 MB of plane) and with the default single group, interleaved over rounds. Prints per-step kernel times (sum of
the launches in one step). Timing only: every setting computes the same records (checked against the first).

usage: python probes/k2_mall_probe.py [rounds]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "audio-ident_amd"))


def run(eng, pcm, offs, steps=30):
    import torch

    for _ in range(10):
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
            **{k: round(ms / steps, 4) for k, (ms, n) in prof.items() if n},
            "launches_per_step": {k: n // steps for k, (ms, n) in prof.items() if n}}


def main():
    import torch

    from aidfp.engine import Engine

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    eng = Engine(44100, device=0)
    n, clips = 441000, 256
    rows = 858  # frames of a 10 s clip at hop 512
    pcm = torch.empty(clips * n, dtype=torch.float32, device="cuda")
    offs = np.arange(clips + 1, dtype=np.int64) * n
    tracks = np.arange(clips, dtype=np.uint32)
    out = {}
    for name, fmax in (("band_limited", 8000), ("full_band", 20000)):
        eng.synth(pcm.data_ptr(), tracks + (0 if fmax == 8000 else 500000), np.zeros(clips, np.int64), n, fmax_hz=fmax)
        ref = None
        for r in range(rounds):
            for per in (0, 64, 32, 16):
                eng.force("plane_rows", per * rows)
                res = run(eng, pcm, offs)
                recs = [eng.hashes(c) for c in range(0, clips, 15)]
                if ref is None:
                    ref = recs
                res["records_equal"] = all(np.array_equal(a, b) for a, b in zip(recs, ref))
                out.setdefault(f"{name}/{per or 'one group'}", []).append(res)
        eng.force("plane_rows", 0)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
