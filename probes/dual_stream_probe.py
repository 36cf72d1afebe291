#!/usr/bin/env python3
"""Timing-only probe for the K1/K2 overlap (option (a) "K1/K2 fusion"): can K2 of one half of the
batch run beside K1 of the other half? The default K1 takes 16 waves and 160,768 B of LDS per CU, so nothing runs
beside it; a 12-wave K1 (the AID_K1_WAVES=12 build of commit 2556354; the knob was resolved to 16 afterwards:
125,824 B, 3 waves per SIMD at 122 VGPRs) leaves room for one K2
workgroup (21 KB, 124 VGPRs) per CU. The probe runs the bench's 256 x 10 s batch as
  single: one engine, one stream, 256 clips per step (the bench's step);
  dual:   two engines on two streams, 128 clips each, issued alternately, so engine B's K1 can overlap engine A's K2/K3;
  alt:    whole 256-clip steps alternating between two engines on two streams (one step's kernel tails overlap the
          next step's first kernels);
and reports ms per step (256 clips) for each, after the bench's clock settle. The records of both modes must be equal.

    python probes/dual_stream_probe.py [--steps 40]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))

SR, CLIPS, CLIP_S = 44100, 256, 10


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    args = ap.parse_args()
    import torch

    from aidfp.engine import Engine

    torch.cuda.set_device(0)
    n = SR * CLIP_S
    pcm = torch.empty(CLIPS * n, dtype=torch.float32, device="cuda")
    a, b = Engine(SR, device=0), Engine(SR, device=0)
    a.synth(pcm.data_ptr(), np.arange(CLIPS, dtype=np.uint32), np.zeros(CLIPS, np.int64), n)
    torch.cuda.synchronize()
    offs = np.arange(CLIPS + 1, dtype=np.int64) * n
    half = CLIPS // 2
    offs_a, offs_b = offs[: half + 1], offs[half:]
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def single(k):
        for _ in range(k):
            a.extract_device(pcm.data_ptr(), offs, sa.cuda_stream)
        torch.cuda.synchronize()

    def dual(k):
        for _ in range(k):
            a.extract_device(pcm.data_ptr(), offs_a, sa.cuda_stream)
            b.extract_device(pcm.data_ptr(), offs_b, sb.cuda_stream)
        torch.cuda.synchronize()

    def alt(k):  # whole steps alternating between two engines on two streams: kernel tails of one step overlap
        for i in range(k):  # the next step's first kernels
            if i % 2 == 0:
                a.extract_device(pcm.data_ptr(), offs, sa.cuda_stream)
            else:
                b.extract_device(pcm.data_ptr(), offs, sb.cuda_stream)
        torch.cuda.synchronize()

    def timed(fn, k):
        t = time.perf_counter()
        fn(k)
        return (time.perf_counter() - t) / k * 1e3

    out = {"k1_waves_per_cu": None, "rounds": []}
    for fn in (single, dual, alt):  # warm-up + clock settle
        fn(4)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.2:
        single(10)
    for _ in range(3):
        out["rounds"].append({"single_ms": round(timed(single, args.steps), 4), "dual_ms": round(timed(dual, args.steps), 4),
                              "alt_ms": round(timed(alt, args.steps), 4)})
    single(1)
    ref = [a.hashes(c) for c in range(CLIPS)]
    dual(1)
    got = [a.hashes(c) for c in range(half)] + [b.hashes(c) for c in range(CLIPS - half)]
    out["records_equal"] = all(np.array_equal(x, y) for x, y in zip(ref, got))
    out["single_ms"] = min(r["single_ms"] for r in out["rounds"])
    out["dual_ms"] = min(r["dual_ms"] for r in out["rounds"])
    out["alt_ms"] = min(r["alt_ms"] for r in out["rounds"])
    alt(2)
    got_alt = [b.hashes(c) for c in range(CLIPS)]
    out["records_equal_alt"] = all(np.array_equal(x, y) for x, y in zip(ref, got_alt))
    out["audio_s_per_s_single"] = round(CLIPS * CLIP_S / out["single_ms"] * 1e3, 1)
    out["audio_s_per_s_dual"] = round(CLIPS * CLIP_S / out["dual_ms"] * 1e3, 1)
    a.close()
    b.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
