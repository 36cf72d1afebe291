#!/usr/bin/env python3
"""K4 index build A/B on the config-3 catalog: hand-written radix sort vs rocPRIM vs the atomic build.

    python probes/k4_probe.py [--tracks 100000] [--reps 3]

Ingests the synthetic catalog once (aidfp.catalog.ingest_synthetic, 1 GPU), then rebuilds the CSR with each
build (aid_engine_force K4_BUILD) and times aid_index_finalize on the host and with the engine's
AID_K_INDEX_BUILD events (sort + bucket lengths + offsets). Run it under `rocprofv3 --kernel-trace --stats`
for the per-kernel split. Prints one JSON line."""
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
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="radix,rocprim,atomic,radix_again",
                    help="builds to time, of radix, rocprim, atomic, radix_again, radix_ballot (the ballot-matched "
                         "in-wave rank) (AIDFP_LIB picks an A/B library)")
    args = ap.parse_args()
    import torch

    from aidfp.catalog import ingest_synthetic
    from aidfp.engine import Engine

    torch.cuda.set_device(0)
    eng = Engine(44100, device=0)
    st = ingest_synthetic(eng, np.arange(args.tracks, dtype=np.uint32), 30.0, batch=1024)
    import os

    out = {"postings": st.postings_total, "library": os.environ.get("AIDFP_LIB", "product")}
    ref = None
    modes = [m for m in (("radix", 1), ("rocprim", 3), ("atomic", 2), ("radix_again", 1), ("radix_ballot", 4))
             if m[0] in args.modes.split(",")]
    for name, mode in modes:
        eng.force("k4_build", mode)
        times, ev = [], []
        for _ in range(args.reps):
            eng.force("k4_build", mode)  # marks the index dirty: the next finalize rebuilds
            eng.profile_enable(True)
            eng.profile_read(reset=True)
            torch.cuda.synchronize()
            t = time.perf_counter()
            eng.index_finalize()
            times.append(time.perf_counter() - t)
            p = eng.profile_read(reset=True)
            eng.profile_enable(False)
            ev.append(p["index_build"][0])
        stats = eng.index_stats()
        # the same index either way: compare a sample of rows of the CSR through queries of random records
        if ref is None:
            ref = stats
        out[name] = {"host_ms": [round(1e3 * x, 2) for x in times], "event_ms": [round(x, 2) for x in ev],
                     "live": stats["live"], "same_live_as_radix": stats["live"] == ref["live"],
                     "bytes_per_posting_at_event_time": None}
    n = st.postings_total
    for name in ("radix", "rocprim"):
        if name not in out:
            continue
        best = min(out[name]["event_ms"])
        out[name]["best_event_ms"] = best
        out[name]["gb_per_s_at_92B" if name == "radix" else "gb_per_s_at_125B"] = round(
            n * (92 if name == "radix" else 125) / (best * 1e-3) / 1e9, 1)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
