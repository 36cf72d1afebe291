#!/usr/bin/env python3
"""bench_resample.py -- K6 `resample` (PCM front-end, FPSPEC 8) on one MI355X.

Workload: 256 x 10 s of 48 kHz interleaved stereo resident in HBM (the UI's capture format,
AudioRecorder.svelte:86-106) -> mono at the index rate: 16 kHz (the reference's Olaf rate,
fingerprint.py:10) and 44.1 kHz (the bench index rate). One step = one aid_resample launch
over the whole batch as one long signal. Roofline: algorithmic HBM bytes per launch
(8 B per stereo input frame read once + 4 B per output written once) / the launch's mean
device time from HIP events (aid_profile_*), against 8.0 TB/s. cpu_baseline: the C oracle
(oracle/fp_resample.c, bit-exact) on one host thread over a 20 s sample.
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))
HBM_PEAK_GBS = 8000.0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--clips", type=int, default=256)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import torch

    from aidfp.engine import Engine

    sr_in = 48000
    n = int(args.clips * args.seconds * sr_in)
    eng = Engine(16000)
    g = torch.Generator(device="cuda").manual_seed(0)
    src = (torch.rand(2 * n, generator=g, device="cuda") - 0.5) * 0.6
    out = []
    for sr_out in (16000, 44100):
        m = eng.resample_len(n, sr_in, sr_out)
        dst = torch.empty(m, dtype=torch.float32, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(args.warmup):
            eng.resample(src.data_ptr(), n, 2, sr_in, sr_out, dst.data_ptr(), m, s)
        torch.cuda.synchronize()
        eng.profile_enable(True)
        eng.profile_read(reset=True)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eng.resample(src.data_ptr(), n, 2, sr_in, sr_out, dst.data_ptr(), m, s)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        ms, cnt = eng.profile_read(reset=True)["resample"]
        eng.profile_enable(False)
        k_ms = ms / cnt
        alg = 8 * n + 4 * m
        up, down, hl, J = eng.resample_plan(sr_in, sr_out)
        cpu = None
        if not args.no_cpu:
            sys.path.insert(0, str(ROOT / "oracle"))
            import oracle as O  # CPU baseline only

            xs = src[: 2 * 20 * sr_in].view(-1, 2).cpu().numpy()
            t = time.perf_counter()
            O.resample(xs, sr_in, sr_out)
            dt = time.perf_counter() - t
            cpu = {"value": round(20.0 / dt, 1), "unit": "audio-s/s", "cores": 1, "kind": "port",
                   "sample": "20 s of the same 48 kHz stereo through oracle/fp_resample.c (-O2, 1 thread)"}
        out.append({
            "metric": f"48 kHz stereo -> {sr_out} Hz mono resampling, audio-s/s per GPU",
            "value": round(args.steps * n / sr_in / wall, 1), "unit": "audio-s/s", "n_gpus": 1,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 4),
            "higher_is_better": True, "dtype": "f32", "data": "synthetic (uniform noise, generated in HBM)",
            "config": {"workload": f"{args.clips} x {args.seconds:g} s 48 kHz stereo as one signal",
                       "up": up, "down": down, "taps_per_phase": J},
            "kernel_ms": round(k_ms, 4),
            "roofline": {"kernel": "resample", "bound": "hbm", "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "algorithmic_bytes_per_launch": alg, "traffic": None},
            "cpu_baseline": cpu,
        })
    for line in out:
        print(json.dumps(line), flush=True)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
