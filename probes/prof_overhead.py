"""Timing-only probe: bench.py's extraction loop with and without the per-kernel profiler events,
alternating in one process (what the event packets cost the step)."""
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "audio-ident_amd"))
from aidfp.engine import Engine  # noqa: E402

SR, CLIPS, CLIP_S, K = 44100, 256, 10, 30
eng = Engine(SR, device=0)
n = SR * CLIP_S
pcm = torch.empty(CLIPS * n, dtype=torch.float32, device="cuda")
eng.synth(pcm.data_ptr(), np.arange(CLIPS, dtype=np.uint32), np.zeros(CLIPS, np.int64), n)
offs = np.arange(CLIPS + 1, dtype=np.int64) * n
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    eng.extract_device(pcm.data_ptr(), offs, s)
torch.cuda.synchronize()
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 3
for rep in range(REPS):
    for prof, sel in ((False, None), (True, None), (True, (0, 1)), (True, (0,))):
        eng.profile_select(sel)
        eng.profile_enable(prof)
        eng.profile_read(reset=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            eng.extract_device(pcm.data_ptr(), offs, s)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K
        p = eng.profile_read(reset=True)
        ks = {k: round(ms / c, 4) for k, (ms, c) in p.items() if c}
        print(f"prof={prof} sel={sel} ms/step {dt * 1e3:.4f} audio-s/s {CLIPS * CLIP_S / dt:.0f} {ks}", flush=True)
