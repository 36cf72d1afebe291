"""Probe: K1/K2/K3 time per block of 20 extraction steps over ~1 s of back-to-back blocks,
to see whether the first blocks after start-up run slower (clock / power-state ramp).
Timing only. usage: python probes/ramp_probe.py [blocks] [sleep_ms]"""
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
    blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    sleep_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
    torch.cuda.set_device(0)
    eng = Engine(SR, device=0)
    n = SR * CLIP_S
    pcm = torch.empty(CLIPS * n, dtype=torch.float32, device="cuda")
    eng.synth(pcm.data_ptr(), np.arange(CLIPS, dtype=np.uint32), np.zeros(CLIPS, np.int64), n)
    stream = torch.cuda.current_stream().cuda_stream
    offs = np.arange(CLIPS + 1, dtype=np.int64) * n
    for _ in range(3):
        eng.extract_device(pcm.data_ptr(), offs, stream)
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for b in range(blocks):
        if sleep_ms and b == blocks // 2:
            time.sleep(sleep_ms / 1e3)
        eng.profile_enable(True)
        eng.profile_read(reset=True)
        t0 = time.perf_counter()
        for _ in range(20):
            eng.extract_device(pcm.data_ptr(), offs, stream)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        prof = eng.profile_read(reset=True)
        eng.profile_enable(False)
        k = {name: round(ms / cnt, 4) for name, (ms, cnt) in prof.items() if cnt}
        print(json.dumps({"block": b, "t_ms": round((t0 - t_start) * 1e3, 1), "ms_per_step": round(dt * 1e3, 4),
                          "M": round(CLIPS * CLIP_S / dt / 1e6, 3), **k}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
