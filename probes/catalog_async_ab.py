#!/usr/bin/env python3
"""Catalog-ingest A/B of the asynchronous posting append: bench.py's catalog leg shape (T synthetic tracks x 30 s,
1,024-track batches, generated on the device and fingerprinted on one stream), with the engine library named by
AIDFP_LIB. --wait-synth keeps the generation synchronous (a library without AID_SYNTH_ASYNC needs it). Prints the
ingest phase as catalog_leg prices it (wall minus the generation's device time), the generation time, the posting
count and the stored postings' checksum (the same for both libraries when the appends agree). Diagnostic only.

    AIDFP_LIB=probes/ab/libaidfp_r05base.so python probes/catalog_async_ab.py --wait-synth
    python probes/catalog_async_ab.py
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=100000)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--wait-synth", action="store_true")
    ap.add_argument("--sr", type=int, default=16000)
    ap.add_argument("--batch", type=int, default=1024, help="tracks per extraction call")
    ap.add_argument("--profile", action="store_true", help="one more pass with the engine's per-kernel events")
    args = ap.parse_args()
    import torch

    from aidfp.engine import Engine

    torch.cuda.set_device(0)
    eng = Engine(args.sr, device=0)
    n = int(round(args.seconds * args.sr)) & ~1
    batch = args.batch
    pcm = torch.empty(batch * n, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    tracks = np.arange(args.tracks, dtype=np.uint32)
    for rep in range(args.reps + 1 + args.profile):
        prof = args.profile and rep == args.reps + 1
        if prof:
            eng.profile_enable(True)
            eng.profile_read(reset=True)
        eng.index_reset()
        ev = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for b0 in range(0, len(tracks), batch):
            tr = tracks[b0:b0 + batch]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            if args.wait_synth:
                eng.synth(pcm.data_ptr(), tr, np.zeros(len(tr), np.int64), n, stream=s.cuda_stream)
            else:
                eng.synth(pcm.data_ptr(), tr, np.zeros(len(tr), np.int64), n, stream=s.cuda_stream, wait=False)
            b.record(s)
            ev.append((a, b))
            eng.extract_device(pcm.data_ptr(), np.arange(len(tr) + 1, dtype=np.int64) * n, s.cuda_stream)
            eng.index_add_extracted(tr)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        t_synth = sum(a.elapsed_time(b) for a, b in ev) * 1e-3
        post = eng.index_stats()["postings"]
        if rep == 0:
            continue  # warm-up (first growth of the planes, allocator)
        if prof:
            k = {name: round(ms, 2) for name, (ms, cnt) in eng.profile_read(reset=True).items() if cnt}
            print(json.dumps({"sr": args.sr, "wall_s": round(wall, 4), "kernel_ms_total": k}), flush=True)
            continue
        print(json.dumps({"lib": "AIDFP_LIB" in __import__("os").environ and "base" or "tree", "sr": args.sr,
                          "wait_synth": args.wait_synth, "batch": batch, "rep": rep, "wall_s": round(wall, 4),
                          "synth_s": round(t_synth, 4), "ingest_s": round(wall - t_synth, 4),
                          "audio_s_per_s": round(args.tracks * args.seconds / (wall - t_synth), 1),
                          "postings": post, "checksum": hex(eng.index_checksum())}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
