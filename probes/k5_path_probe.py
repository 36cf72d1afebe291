#!/usr/bin/env python3
"""K5 path A/B on the config-4 workload: the exact lane over the 100k-track catalog with the engine's own path choice
(auto), the LDS vote table forced first (k5_path 1), and the global histogram forced (k5_path 2). Rows must agree.

    python probes/k5_path_probe.py [--tracks 100000] [--clips 4096] [--reps 3]"""
import argparse
import json
import sys
import time
import types
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))
sys.path.insert(0, str(ROOT))


def reps_or1(args):
    return max(1, args.reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=100000)
    ap.add_argument("--clips", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--paths", default="auto,lds_first,global,auto_again")
    args = ap.parse_args()
    import torch

    from aidfp import synth
    from aidfp.catalog import ingest_synthetic
    from aidfp.engine import Engine

    SR = 44100
    torch.cuda.set_device(0)
    eng = Engine(SR, device=0)
    ingest_synthetic(eng, np.arange(args.tracks, dtype=np.uint32), 30.0, batch=1024)
    eng.index_finalize()
    rng = np.random.default_rng(5)
    n = args.clips
    truth = rng.integers(0, args.tracks, n).astype(np.uint32)
    starts = rng.integers(0, 25 * SR, n).astype(np.int64)
    clip_n = 5 * SR
    pcm = torch.empty(n * clip_n, dtype=torch.float32, device="cuda")
    eng.synth(pcm.data_ptr(), truth, starts, clip_n, noise_a=synth.noise_halfwidth(20.0), salt=77)
    pcm.mul_(0.5)
    offs = np.arange(n + 1, dtype=np.int64) * clip_n
    out = {"tracks": args.tracks, "clips": n}
    ref = None
    codes = {"auto": 0, "lds_first": 1, "global": 2, "auto_again": 0, "auto_gather": 0}
    for name in args.paths.split(","):
        path = codes[name]
        eng.force("k5_path", path)
        eng.force("lane_gather", int(name == "auto_gather"))  # sub-windows staged (A/B) or read in place
        eng.exact_lane(pcm_ptr=pcm.data_ptr(), offsets=offs, max_out=10)  # warm
        eng.match_stats(reset=True)
        ts = []
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rows = eng.exact_lane(pcm_ptr=pcm.data_ptr(), offsets=offs, max_out=10)
            ts.append(time.perf_counter() - t)
        ms = eng.match_stats(reset=True)
        eng.profile_enable(True)
        eng.profile_read(reset=True)
        eng.exact_lane(pcm_ptr=pcm.data_ptr(), offsets=offs, max_out=10)  # untimed: per-kernel times
        prof = eng.profile_read(reset=True)
        eng.profile_enable(False)
        eng.match_stats(reset=True)
        k5_ms = sum(prof[k][0] for k in ("match", "vote_hist", "hot_scan", "vote_final") if k in prof)
        top1 = float(np.mean([len(r) > 0 and int(r[0]["track"]) == int(t) for r, t in zip(rows, truth)]))
        same = True
        if ref is None:
            ref = rows
        else:
            same = all(np.array_equal(a, b) for a, b in zip(ref, rows))
        out[name] = {"s": [round(x, 4) for x in ts], "clips_per_s": round(n / min(ts), 1), "top1": top1,
                     "rows_equal_auto": same, "votes_per_query": round(ms["votes"] / max(1, ms["queries"]), 1),
                     "queries_lds": ms["queries_lds"], "queries_global": ms["queries_global"],
                     "k5_ms": round(k5_ms, 3), "k5_frac": round(8 * ms["votes"] / reps_or1(args) / k5_ms / 8e9, 4) if k5_ms else None}
        print(json.dumps({name: out[name]}), file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
