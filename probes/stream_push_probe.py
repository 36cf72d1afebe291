"""Where one streaming push's latency goes (bench_stream.py, BASELINE config 5): host->device copy, downmix,
window assembly, extraction, query. Synchronises after every stage (so the stages add up to more than a
normal push). Diagnostic only. usage: python probes/stream_push_probe.py
"""
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "audio-ident_amd"))


def main():
    import torch

    from aidfp import synth
    from aidfp.catalog import ingest_synthetic
    from aidfp.engine import Engine

    SR = 48000
    eng = Engine(SR, device=0)
    ingest_synthetic(eng, np.arange(200, dtype=np.uint32), 30.0)
    chunk = int(2.5 * SR)
    x = np.stack([synth.synth(3, 0, chunk, SR, salt=1), synth.synth(3, 0, chunk, SR, salt=2)], axis=1)
    win = 5 * SR
    stage = torch.empty(2 * chunk, dtype=torch.float32, device="cuda")
    mono = torch.zeros(4 * win, dtype=torch.float32, device="cuda")
    wbuf = torch.empty(win, dtype=torch.float32, device="cuda")
    pinned = torch.empty(2 * chunk, dtype=torch.float32).pin_memory()
    s = torch.cuda.current_stream().cuda_stream
    t = {k: [] for k in ("h2d_pageable", "h2d_pinned", "downmix", "window", "extract", "query")}
    for it in range(60):
        torch.cuda.synchronize()
        a = time.perf_counter()
        stage.copy_(torch.from_numpy(x.reshape(-1)))
        torch.cuda.synchronize()
        b = time.perf_counter()
        pinned.numpy()[:] = x.reshape(-1)
        stage.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        c = time.perf_counter()
        eng.downmix(stage.data_ptr(), chunk, mono.data_ptr(), s)
        torch.cuda.synchronize()
        d = time.perf_counter()
        wbuf.copy_(mono[:win])
        torch.cuda.synchronize()
        e = time.perf_counter()
        eng.extract_device(wbuf.data_ptr(), np.array([0, win], np.int64), s)
        eng.sync()
        f = time.perf_counter()
        eng.query_extracted()
        g = time.perf_counter()
        if it >= 10:
            for k, v in zip(t, (b - a, c - b, d - c, e - d, f - e, g - f)):
                t[k].append(v)
    print(json.dumps({k: round(1e3 * float(np.median(v)), 4) for k, v in t.items()}))


if __name__ == "__main__":
    main()
