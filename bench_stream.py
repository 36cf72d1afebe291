#!/usr/bin/env python3
"""BASELINE config 5: 48 kHz stereo streaming, 50 %-overlap 5 s windows, continuous
identification on 1 GPU.

A 10-minute synthetic stream is the concatenation of 30 s segments of catalog
tracks (left/right = the same track with independent noise at SNR 30 dB). It is
pushed in real-time-sized chunks (default 2.5 s = one window hop) through
aidfp.stream.StreamIdentifier: GPU downmix -> window -> K1-K3 -> K5 against a
48 kHz index. Reports sustained audio-s/s (stream time / processing time),
per-push latency percentiles, and top-1 accuracy over windows that lie inside a
single segment.
"""

from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent / "audio-ident_amd"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=1000)
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--chunk-s", type=float, default=2.5)
    ap.add_argument("--index-sr", type=int, default=48000,
                    help="index rate; != 48000 resamples the stream on the GPU (16000 = the reference's Olaf rate)")
    ap.add_argument("--source-sr", type=int, default=44100,
                    help="rate the catalog tracks are synthesised at before K6 brings them to --index-sr, as ingest "
                         "decodes each file with ffmpeg -ar (decode.py:41-60); 0 = synthesise at the index rate")
    args = ap.parse_args()
    SR = 48000
    ISR = args.index_sr
    import torch

    from aidfp import synth
    from aidfp.catalog import ingest_synthetic
    from aidfp.engine import Engine
    from aidfp.stream import StreamIdentifier

    torch.cuda.set_device(0)
    eng = Engine(ISR, device=0)
    ingest_synthetic(eng, np.arange(args.tracks, dtype=np.uint32), 30.0, source_sr=args.source_sr or None)
    rng = np.random.default_rng(42)
    seg = 30 * SR
    n_seg = int(args.minutes * 60 / 30)
    seg_tracks = rng.integers(0, args.tracks, n_seg)
    left = np.concatenate([synth.synth(int(t), 0, seg, SR, snr_db=30.0, salt=11) for t in seg_tracks])
    right = np.concatenate([synth.synth(int(t), 0, seg, SR, snr_db=30.0, salt=12) for t in seg_tracks])
    stereo = np.stack([left, right], axis=1)

    sid = StreamIdentifier(eng, stream_sr=SR)
    chunk = int(args.chunk_s * SR)
    lat = []
    results = []
    sid.push(stereo[:chunk])  # warm-up (first allocations)
    sid = StreamIdentifier(eng, stream_sr=SR)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for a in range(0, len(stereo), chunk):
        t = time.perf_counter()
        results += sid.push(stereo[a:a + chunk])
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t)
    total = time.perf_counter() - t0
    ok = n = 0
    for r in results:
        s0 = int(round(r.start_s * SR))
        si, sj = s0 // seg, (s0 + int(round(sid.win * SR / ISR)) - 1) // seg
        if si != sj:
            continue
        n += 1
        ok += r.best_track == int(seg_tracks[si])
    stream_s = len(stereo) / SR
    print(json.dumps({
        "metric": "48 kHz stereo stream, 5 s / 2.5 s windows: sustained audio-s/s, 1 GPU",
        "index_sr": ISR, "index_source_sr": args.source_sr or ISR, "front_end": "downmix" if ISR == SR else f"downmix + resample 48000 -> {ISR} (K6)",
        "value": round(stream_s / total, 1), "unit": "audio-s/s", "n_gpus": 1,
        "stream_s": stream_s, "windows": len(results), "chunk_s": args.chunk_s,
        "push_latency_ms": {p: round(1e3 * float(np.percentile(lat, q)), 3) for p, q in (("p50", 50), ("p95", 95), ("p99", 99))},
        "top1_windows_inside_segment": round(ok / max(1, n), 4), "index_tracks": args.tracks, "data": "synthetic",
    }), flush=True)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
