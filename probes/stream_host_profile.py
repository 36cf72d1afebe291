#!/usr/bin/env python3
"""Where a StreamBank push spends its host time (bench.py's stream leg shape: S live 48 kHz stereo streams, 2.5 s
pushes, a 16 kHz index from 44.1 kHz sources): the push's wall time, the GPU kernels' time per push from the engine's
HIP-event profile, and cProfile's top functions over the timed pushes. Diagnostic only.

    python probes/stream_host_profile.py [--streams 256] [--tracks 1000] [--seconds 60]
"""
import argparse
import cProfile
import io
import json
import pstats
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=256)
    ap.add_argument("--tracks", type=int, default=1000)
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--pipelined", action="store_true", help="push_submit N + 1 then collect N (bench's pipelined loop)")
    args = ap.parse_args()
    import torch

    from aidfp import synth
    from aidfp.catalog import ingest_synthetic
    from aidfp.engine import Engine
    from aidfp.stream import StreamBank

    torch.cuda.set_device(0)
    SSR, QSR, S = 16000, 48000, args.streams
    eng = Engine(SSR, device=0)
    ingest_synthetic(eng, np.arange(args.tracks, dtype=np.uint32), 30.0, batch=1024, source_sr=44100, local=True)
    eng.index_finalize()
    n = int(args.seconds * QSR)
    seg = 30 * QSR
    n_seg = max(1, n // seg)
    rng = np.random.default_rng(5)
    tr = rng.integers(0, args.tracks, (S, n_seg)).astype(np.uint32)
    stereo = torch.empty(S, n_seg * seg, 2, dtype=torch.float32, device="cuda")
    tmp = torch.empty(S * n_seg * seg, dtype=torch.float32, device="cuda")
    for ch in range(2):
        eng.synth(tmp.data_ptr(), tr.ravel(), np.zeros(S * n_seg, np.int64), seg, noise_a=synth.noise_halfwidth(30.0),
                  salt=11 + ch, sample_rate=QSR)
        stereo[:, :, ch] = tmp.view(S, n_seg * seg)
    del tmp
    chunk = int(2.5 * QSR)

    def run(prof=None, gpu=False):
        bank = StreamBank(eng, S, stream_sr=QSR)
        bank.timings = []
        if gpu:
            eng.profile_enable(True)
            eng.profile_read(reset=True)
        torch.cuda.synchronize()
        lat, split = [], []
        pending = None
        for a in range(0, stereo.shape[1], chunk):
            t = time.perf_counter()
            if prof:
                prof.enable()
            if args.pipelined:
                p = bank.push_submit(stereo[:, a:a + chunk])
                t1 = time.perf_counter()
                if pending is not None:
                    pending.collect()
                pending = p
                split.append((t1 - t, time.perf_counter() - t1))
            else:
                bank.push(stereo[:, a:a + chunk])
            if prof:
                prof.disable()
            lat.append(time.perf_counter() - t)
        if pending is not None:
            pending.collect()
        torch.cuda.synchronize()
        if split:
            bank.timings = [tuple(x) + (sb, cl) for x, (sb, cl) in zip(bank.timings, split)]
        kern = None
        if gpu:
            kern = {k: round(ms / len(lat), 4) for k, (ms, cnt) in eng.profile_read(reset=True).items() if cnt}
            eng.profile_enable(False)
        return lat, bank.timings, kern

    run()  # warm-up
    lat, tim, _ = run()
    _, _, kern = run(gpu=True)
    prof = cProfile.Profile()
    run(prof)
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(18)
    tim = np.array(tim)
    print(json.dumps({"streams": S, "pipelined": args.pipelined, "push_ms_p50": round(1e3 * float(np.median(lat)), 3),
                      # pipelined: + submit call, collect call
                      "append_resample_windows_ms_p50": [round(1e3 * float(np.median(tim[:, i])), 3)
                                                         for i in range(tim.shape[1])],
                      "gpu_ms_per_push_by_kernel_group": kern}), flush=True)
    print(s.getvalue(), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
