#!/usr/bin/env python3
"""CPU-only probe of the drop-in service's HOST side (the serving path is host-bound).

bench.py's service leg (64 closed-loop `olaf_query` clients on one event loop -> QueryCoalescer -> one engine call
per batch) with the engine call replaced by a stand-in that does the call's host-visible work -- the batch's PCM laid
into page-locked-style staging (the real `_host_concat`), then a GIL-free wait of `--gpu-ms` standing for the H2D copy
and the kernels (time.sleep releases the GIL as the ctypes call does), then the rows of a typical answer. It measures
what the Python layers cost per request and how the dispatcher count changes throughput, with no GPU.

    python probes/service_host_probe.py [--clients 64] [--requests 4096] [--gpu-ms 0.7] [--workers 1 2]
"""
import argparse
import asyncio
import gc
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))

from aidfp import engine as E  # noqa: E402
from aidfp import fingerprint as fp  # noqa: E402


class FakeEngine:
    """The Engine surface FingerprintService._query_batch uses."""

    hop, sample_rate, max_results = 256, 16000, 50

    def __init__(self, gpu_ms: float, rows_per_query: int):
        self.gpu_s = gpu_ms * 1e-3
        self.k = rows_per_query
        self._slot = E._new_slot()

    def close(self):
        pass

    def query_pcm(self, clips):
        arrs = [np.ascontiguousarray(c, dtype=np.float32).ravel() for c in clips]
        total = sum(len(a) for a in arrs)
        E._host_concat(arrs, total)  # the real staging copy
        time.sleep(self.gpu_s)  # the engine call: GIL released (ctypes), H2D + kernels
        return self._answer(clips)

    def query_pcm_submit(self, clips):
        """The pipelined half: the staging copy now; the 'GPU' finishes gpu_ms after the previous submit's work (one
        stream), and collect() sleeps until then."""
        arrs = [np.ascontiguousarray(c, dtype=np.float32).ravel() for c in clips]
        E._host_concat(arrs, sum(len(a) for a in arrs), self._slot)
        now = time.perf_counter()
        self._busy_until = max(now, getattr(self, "_busy_until", 0.0)) + self.gpu_s
        done, out = self._busy_until, self._answer(clips)

        class Pending:
            def collect(self_):
                left = done - time.perf_counter()
                if left > 0:
                    time.sleep(left)
                return out

        return Pending()

    def _answer(self, clips):
        out = []
        for i in range(len(clips)):
            r = np.zeros((self.k, 5), np.int64)
            r[:, 0] = np.arange(200, 200 - self.k, -1)
            r[:, 1] = (i + np.arange(self.k)) % 1000
            out.append(r)
        return out


def run(workers: int, clients: int, n_req: int, gpu_ms: float, rows: int, pipeline: bool = False,
        max_batch: int = 256, split_min: int = 0, split_parts: int = 2) -> dict:
    svc = fp.FingerprintService(Path("/tmp/aidfp_probe_db"), coalesce_workers=workers, pipeline=pipeline,
                                max_batch=max_batch, split_min=split_min, split_parts=split_parts)
    svc.persist = False
    svc._engine = FakeEngine(gpu_ms, rows)
    svc._names = {i: f"track-{i}" for i in range(1000)}
    fp.set_service(svc)
    req = (np.random.default_rng(0).standard_normal(80000).astype("<f4")).tobytes()  # 5 s at 16 kHz
    lat = np.zeros(n_req)
    nxt = [0]

    async def client():
        while nxt[0] < n_req:
            i = nxt[0]
            nxt[0] += 1
            t = time.perf_counter()
            await fp.olaf_query(req)
            lat[i] = time.perf_counter() - t

    async def level():
        await asyncio.gather(*(client() for _ in range(clients)))

    for _ in range(4):
        svc.query(req)
    gc.collect()
    gc.freeze()
    svc._coalescer.batches.clear()
    t0 = time.perf_counter()
    asyncio.run(level())
    wall = time.perf_counter() - t0
    gc.unfreeze()
    b = np.array(svc._coalescer.batches)
    fp.set_service(None)
    svc.close()
    return {"workers": workers, "pipeline": pipeline, "max_batch": max_batch, "split_min": split_min,
            "split_parts": split_parts, "overlapped": svc._coalescer.overlapped,
            "clients": clients, "gpu_ms": gpu_ms, "qps": round(n_req / wall, 1),
            "p50_ms": round(1e3 * float(np.percentile(lat, 50)), 3), "p95_ms": round(1e3 * float(np.percentile(lat, 95)), 3),
            "mean_batch": round(float(b.mean()), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=64)
    ap.add_argument("--requests", type=int, default=4096)
    ap.add_argument("--gpu-ms", type=float, default=0.7)
    ap.add_argument("--rows", type=int, default=3)
    ap.add_argument("--workers", type=int, nargs="+", default=[1, 2])
    ap.add_argument("--pipeline", type=int, nargs="+", default=[0], help="0/1: the coalescer's pipelined dispatch")
    ap.add_argument("--max-batch", type=int, nargs="+", default=[256])
    ap.add_argument("--split-min", type=int, nargs="+", default=[0])
    ap.add_argument("--split-parts", type=int, nargs="+", default=[2])
    ap.add_argument("--profile", action="store_true")
    a = ap.parse_args()
    for w, pl, mb, sm, sp in [(w, pl, mb, sm, sp) for w in a.workers for pl in a.pipeline for mb in a.max_batch
                              for sm in a.split_min for sp in a.split_parts]:
        if a.profile:
            import cProfile
            import pstats

            pr = cProfile.Profile()
            pr.enable()
            r = run(w, a.clients, a.requests, a.gpu_ms, a.rows, bool(pl), mb, sm, sp)
            pr.disable()
            pstats.Stats(pr).sort_stats("tottime").print_stats(18)
        else:
            r = run(w, a.clients, a.requests, a.gpu_ms, a.rows, bool(pl), mb, sm, sp)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
