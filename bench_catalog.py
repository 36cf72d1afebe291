#!/usr/bin/env python3
"""BASELINE config 3: synthetic catalog ingest sharded across the GPUs of one node.

    python bench_catalog.py --tracks 100000 --seconds 30                # 1 GPU
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench_catalog.py --tracks 100000            # 8 GPUs

Each rank generates its shard of tracks in HBM (aid_synth), fingerprints it
(K1-K3) and appends postings; one RCCL all-gather then replicates every rank's
postings and each GPU builds the full CSR index (K4). Prints one JSON line:
audio-seconds ingested per second for the whole job, phase times (max over
ranks) and a top-1 spot check of the replicated index on rank 0.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent / "audio-ident_amd"))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tracks", type=int, default=100000)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--sr", type=int, default=44100)
    ap.add_argument("--check", type=int, default=64, help="spot-check queries on rank 0")
    ap.add_argument("--exchange", choices=("native", "torch"), default="native",
                    help="native: aid_index_allgather over the engine's RCCL comm; torch: torch.distributed")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    rank = dist.get_rank() if world > 1 else 0

    from aidfp import synth
    from aidfp.catalog import ingest_synthetic
    from aidfp.engine import Engine

    eng = Engine(args.sr, device=local)
    tracks = np.arange(args.tracks, dtype=np.uint32)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    st = ingest_synthetic(eng, tracks, args.seconds, batch=args.batch, exchange=args.exchange)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    # the synthetic tracks are generated on the device inside the extract span (SURVEY 8d config 3:
    # "generated on device"); the ingest rate excludes that generation time, wall_s keeps it
    phases = torch.tensor([wall - st.t_synth, st.t_extract - st.t_synth, st.t_exchange, st.t_build, st.t_comm_init,
                           st.t_synth, wall], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(phases, op=dist.ReduceOp.MAX)
    ingest, te, tx, tb, ti, tsyn, wall = phases.tolist()

    acc = None
    if rank == 0 and args.check:
        rng = np.random.default_rng(42)
        tr = rng.integers(0, args.tracks, size=args.check)
        starts = rng.integers(0, int((args.seconds - 5) * args.sr), size=args.check)
        clips = [synth.synth(int(t), int(s), 5 * args.sr, args.sr, snr_db=20.0, salt=3) for t, s in zip(tr, starts)]
        eng.extract_host(clips)
        rows = eng.query_extracted()
        acc = float(np.mean([len(r) > 0 and r[0, 1] == t for r, t in zip(rows, tr)]))

    if rank == 0:
        audio = args.tracks * args.seconds
        print(json.dumps({
            "metric": "catalog ingest audio-seconds/sec (extract + RCCL all-gather + index build), whole job",
            "value": round(audio / ingest, 1), "unit": "audio-s/s", "n_gpus": world, "tracks": args.tracks,
            "track_seconds": args.seconds, "ingest_s": round(ingest, 3), "wall_s_with_generation": round(wall, 3),
            "synth_generation_s": round(tsyn, 3),
            "phase_s_max_over_ranks": {"extract": round(te, 3), "allgather": round(tx, 3), "build": round(tb, 3),
                                       "comm_init": round(ti, 3)},
            "exchange": st.exchange,
            "postings_total": st.postings_total, "index_bytes_per_gpu": st.postings_total * 8 + (2**26 + 1) * 4,
            "top1_spot_check": acc, "data": "synthetic (aid_synth, generated in HBM)",
        }), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
