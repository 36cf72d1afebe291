"""Probe: one extraction call over 256 x 10 s clips against G calls over 256/G clips each.

Since K1 stores only hot 64-bin blocks (~0.27 GB per 256 clips on the bench data), a group of
128 clips writes ~137 MB, which fits the 256 MB Infinity Cache: K2 may then read K1's output
from the MALL instead of HBM. Earlier group experiments ("Pipelining K1 -> K2") wrote
the full power plane. Timing only (later groups overwrite earlier groups' records).

usage: python probes/group_probe.py [reps]
"""
import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))
from aidfp.engine import Engine  # noqa: E402

SR, CLIPS, CLIP_S = 44100, 256, 10


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    torch.cuda.set_device(0)
    eng = Engine(SR, device=0)
    n = SR * CLIP_S
    pcm = torch.empty(CLIPS * n, dtype=torch.float32, device="cuda")
    eng.synth(pcm.data_ptr(), np.arange(CLIPS, dtype=np.uint32), np.zeros(CLIPS, np.int64), n)
    stream = torch.cuda.current_stream().cuda_stream
    res = {}
    for r in range(reps):
        for G in (1, 2, 4):
            per = CLIPS // G
            offs = np.arange(per + 1, dtype=np.int64) * n
            ptrs = [pcm.data_ptr() + g * per * n * 4 for g in range(G)]
            for _ in range(3):
                for p in ptrs:
                    eng.extract_device(p, offs, stream)
            torch.cuda.synchronize()
            eng.profile_enable(True)
            eng.profile_read(reset=True)
            steps = 20
            t0 = time.perf_counter()
            for _ in range(steps):
                for p in ptrs:
                    eng.extract_device(p, offs, stream)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            prof = eng.profile_read(reset=True)
            eng.profile_enable(False)
            k = {name: round(ms / cnt * G, 4) for name, (ms, cnt) in prof.items() if cnt}
            res.setdefault(G, []).append((round(CLIPS * CLIP_S / dt / 1e6, 3), round(dt * 1e3, 4), k))
            print(json.dumps({"groups": G, "rep": r, "M_audio_s_per_s": res[G][-1][0], "ms_per_step": res[G][-1][1],
                              "kernel_ms_per_step": k}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
