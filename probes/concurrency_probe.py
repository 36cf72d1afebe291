#!/usr/bin/env python3
"""Query latency under concurrency through the drop-in service (SURVEY.md 8b concurrent readers).

    python probes/concurrency_probe.py [--tracks 2000] [--requests 512] [--levels 1,16,64]

Indexes `tracks` synthetic 30 s tracks through FingerprintService.index_track (16 kHz, persist off), then for
each concurrency level c runs c clients that each send queries (5 s clips of indexed tracks at random offsets,
20 dB SNR) back to back until `requests` have completed:
  * "async": c coroutines on one event loop awaiting `olaf_query` (the reference's async API, as a FastAPI
    worker calls it);
  * "threads": c OS threads calling FingerprintService.query (blocking), a harsher GIL load.
Reports per-request latency p50/p99, throughput, the coalescer's batch sizes and the top-1 hit rate. Prints one
JSON line."""
import argparse
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))
SR = 16000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=2000)
    ap.add_argument("--requests", type=int, default=512)
    ap.add_argument("--levels", default="1,16,64")
    ap.add_argument("--clip-s", type=float, default=5.0)
    args = ap.parse_args()
    import tempfile

    from aidfp import fingerprint as fp
    from aidfp import synth

    def pcm(track, start_s, dur_s, snr=None, salt=0):
        return synth.synth(track, int(start_s * SR), int(dur_s * SR), SR, snr_db=snr, salt=salt).astype(
            "<f4").tobytes()

    out = {"tracks": args.tracks, "clip_s": args.clip_s, "sample_rate": SR}
    with tempfile.TemporaryDirectory() as db:
        svc = fp.FingerprintService(Path(db))
        svc.persist = False
        t0 = time.perf_counter()
        for t in range(args.tracks):
            assert svc.index_track(pcm(t, 0, 30.0), f"track-{t}")
        out["index_s"] = round(time.perf_counter() - t0, 2)
        rng = np.random.default_rng(7)
        n = args.requests
        tracks = rng.integers(0, args.tracks, n)
        starts = rng.uniform(0, 30.0 - args.clip_s, n)
        queries = [pcm(int(tr), float(s), args.clip_s, snr=20, salt=i) for i, (tr, s) in enumerate(zip(tracks, starts))]
        for _ in range(8):  # warm the engine buffers for the largest batch shape
            svc.query(queries[0])
        fp.set_service(svc)

        def report(mode, c, lat, hits, wall):
            b = np.array(svc._coalescer.batches)
            e = {"requests": n, "p50_ms": round(1e3 * float(np.percentile(lat, 50)), 2),
                 "p99_ms": round(1e3 * float(np.percentile(lat, 99)), 2),
                 "mean_ms": round(1e3 * float(lat.mean()), 2), "qps": round(n / wall, 1),
                 "batches": int(len(b)), "mean_batch": round(float(b.mean()), 2) if len(b) else 0,
                 "top1": round(float(hits.mean()), 4)}
            out.setdefault(mode, {})[str(c)] = e
            print(json.dumps({"mode": mode, "level": c, **e}), file=sys.stderr, flush=True)

        import asyncio

        for c in [int(x) for x in args.levels.split(",")]:
            lat = np.zeros(n)
            hits = np.zeros(n, dtype=bool)
            nxt = [0]

            async def client():
                while nxt[0] < n:
                    i = nxt[0]
                    nxt[0] += 1
                    t = time.perf_counter()
                    r = await fp.olaf_query(queries[i])
                    lat[i] = time.perf_counter() - t
                    hits[i] = bool(r) and r[0].reference_path == f"track-{int(tracks[i])}"

            async def run_level():
                await asyncio.gather(*(client() for _ in range(c)))

            svc._coalescer.batches.clear()
            t0 = time.perf_counter()
            asyncio.run(run_level())
            report("async", c, lat, hits, time.perf_counter() - t0)
        for c in [int(x) for x in args.levels.split(",")]:
            lat = np.zeros(n)
            hits = np.zeros(n, dtype=bool)
            nxt = [0]
            lock = threading.Lock()

            def client():
                while True:
                    with lock:
                        i = nxt[0]
                        nxt[0] += 1
                    if i >= n:
                        return
                    t = time.perf_counter()
                    r = svc.query(queries[i])
                    lat[i] = time.perf_counter() - t
                    hits[i] = bool(r) and r[0].reference_path == f"track-{int(tracks[i])}"

            svc._coalescer.batches.clear()
            th = [threading.Thread(target=client) for _ in range(c)]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            report("threads", c, lat, hits, time.perf_counter() - t0)
        fp.set_service(None)
        svc.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
