"""Where catalog ingest (bench_catalog.py, BASELINE config 3) spends its wall time per batch:
synth, extraction, index_add_extracted (host syncs + posting-plane growth). Diagnostic only.

usage: python probes/ingest_probe.py [--tracks 100000] [--batch 1024]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "audio-ident_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=100000)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--reserve", type=float, default=0.0, help="postings to reserve up front (0 = none)")
    args = ap.parse_args()
    import torch

    from aidfp.engine import Engine

    eng = Engine(44100, device=0)
    n = int(round(args.seconds * 44100)) & ~1
    pcm = torch.empty(args.batch * n, dtype=torch.float32, device="cuda")
    if args.reserve and hasattr(eng, "index_reserve"):
        eng.index_reserve(int(args.reserve))
    tracks = np.arange(args.tracks, dtype=np.uint32)
    t_syn = t_ext = t_add = 0.0
    worst = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b0 in range(0, args.tracks, args.batch):
        tr = tracks[b0 : b0 + args.batch]
        a = time.perf_counter()
        eng.synth(pcm.data_ptr(), tr, np.zeros(len(tr), np.int64), n)
        torch.cuda.synchronize()
        b = time.perf_counter()
        eng.extract_device(pcm.data_ptr(), np.arange(len(tr) + 1, dtype=np.int64) * n)
        eng.sync()
        c = time.perf_counter()
        eng.index_add_extracted(tr)
        d = time.perf_counter()
        t_syn += b - a
        t_ext += c - b
        t_add += d - c
        worst.append(d - c)
    wall = time.perf_counter() - t0
    print(json.dumps({"tracks": args.tracks, "batch": args.batch, "wall_s": round(wall, 3), "synth_s": round(t_syn, 3),
                      "extract_s": round(t_ext, 3), "index_add_s": round(t_add, 3),
                      "index_add_worst_ms": [round(1e3 * x, 2) for x in sorted(worst)[-8:]],
                      "postings": eng.index_stats()["postings"]}))


if __name__ == "__main__":
    main()
