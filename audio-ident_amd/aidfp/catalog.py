"""Catalog ingest sharded over the GPUs of one node (BASELINE config 3).

The reference ingests one file at a time through a single LMDB writer
(audio-ident-service/app/ingest/pipeline.py:294-310, fingerprint.py:7-8). Here
every rank (one process per GPU) fingerprints its own shard of the tracks
(extraction shards by track, no communication), then ONE exchange replicates
the index: each rank's postings (hash, track, t) are all-gathered over RCCL /
xGMI (torch.distributed "nccl" backend = RCCL on ROCm), so every GPU holds the
whole catalog and can answer queries alone.

RCCL has no all-gatherv: counts are all-gathered first, then every rank's
postings padded to the largest count go through a single all-gather, and the
padding is dropped on receive. Two implementations of that exchange:
  * "native" (default on GPUs): aid_index_allgather in libaidfp over an RCCL
    communicator the engine owns (aid_comm_create; rank 0's unique id is shared
    with broadcast_object_list) -- device postings never leave the C ABI;
  * "torch": `allgather_postings` with torch.distributed collectives. It is
    device-agnostic, so it also runs under gloo on CPU tensors
    (tests/test_catalog_dist.py).
"""

from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np


def shard(tracks, rank: int, world: int):
    """Contiguous block of the track list for `rank` (balanced to within one track)."""
    n = len(tracks)
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return tracks[lo:hi]


def allgather_postings(local, group=None):
    """All-gather variable-length [n, 3] int32 posting blocks; returns [sum n, 3] in rank order."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = local.device
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=dev)
    counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(counts, n, group=group)
    cnt = counts.cpu().tolist()
    mx = max(cnt)
    if mx == 0:
        return local.new_zeros((0, 3))
    send = local.new_zeros((mx, 3))
    send[: local.shape[0]] = local
    recv = local.new_empty((world * mx, 3))
    dist.all_gather_into_tensor(recv, send, group=group)
    recv = recv.view(world, mx, 3)
    return torch.cat([recv[r, : cnt[r]] for r in range(world)], dim=0)


@dataclass
class IngestStats:
    tracks_local: int
    audio_s_local: float
    postings_local: int
    postings_total: int
    t_extract: float
    t_exchange: float
    t_build: float
    exchange: str = "none"
    t_comm_init: float = 0.0
    t_synth: float = 0.0  # device time generating the synthetic PCM (inside t_extract's wall span)


def native_comm(eng, group=None) -> int:
    """aid_comm over the ranks of `group`: rank 0's RCCL id is broadcast through torch.distributed."""
    import torch.distributed as dist

    rank = dist.get_rank(group)
    obj = [eng.comm_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return eng.comm_create(obj[0], dist.get_world_size(group), rank)


def ingest_synthetic(eng, track_ids, seconds: float, batch: int = 512, group=None,
                     exchange: str = "native") -> IngestStats:
    """Fingerprint this rank's shard of synthetic tracks on its GPU, replicate the index.

    `track_ids` is the full catalog (global ids); with torch.distributed initialised
    each rank takes shard(track_ids, rank, world), otherwise the whole list."""
    import torch
    import torch.distributed as dist

    distributed = dist.is_available() and dist.is_initialized()
    rank = dist.get_rank(group) if distributed else 0
    world = dist.get_world_size(group) if distributed else 1
    mine = np.asarray(shard(np.asarray(track_ids, dtype=np.uint32), rank, world), dtype=np.uint32)
    n = int(round(seconds * eng.sample_rate)) & ~1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pcm = torch.empty(max(1, min(batch, len(mine))) * n, dtype=torch.float32, device="cuda")
    base = eng.index_stats()["postings"]
    # one non-default stream for generation, extraction and the posting append: events recorded on
    # the legacy default stream would serialise against the engine's (blocking) stream every batch
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    ev = []
    for b0 in range(0, len(mine), batch):
        tr = mine[b0 : b0 + batch]
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.synth(pcm.data_ptr(), tr, np.zeros(len(tr), np.int64), n, stream=s.cuda_stream)
        b.record(s)
        ev.append((a, b))
        eng.extract_device(pcm.data_ptr(), np.arange(len(tr) + 1, dtype=np.int64) * n, s.cuda_stream)
        eng.index_add_extracted(tr)
    del pcm
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    t_synth = sum(a.elapsed_time(b) for a, b in ev) * 1e-3
    n_local = eng.index_stats()["postings"] - base
    total = n_local
    t_init = 0.0
    if world > 1 and exchange == "native":
        ti = time.perf_counter()
        comm = native_comm(eng, group)
        t1 = time.perf_counter()
        t_init = t1 - ti
        try:
            total = eng.index_allgather(comm, base) - base
        finally:
            eng.comm_destroy(comm)
        t2 = time.perf_counter()
    elif world > 1:
        cols = torch.empty((3, max(n_local, 1)), dtype=torch.int32, device="cuda")
        eng.index_export_device(cols[0].data_ptr(), cols[1].data_ptr(), cols[2].data_ptr(), base, n_local)
        local = cols[:, :n_local].t().contiguous()
        allp = allgather_postings(local, group)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        # replace this rank's postings by the gathered catalog (own shard included, rank order)
        keep = eng.index_export(0, base) if base else None
        eng.index_reset()
        if keep is not None and len(keep):
            k = torch.from_numpy(keep.astype(np.int32)).cuda().t().contiguous()
            eng.index_add_postings(k[0].data_ptr(), k[1].data_ptr(), k[2].data_ptr(), k.shape[1])
        g = allp.t().contiguous()
        eng.index_add_postings(g[0].data_ptr(), g[1].data_ptr(), g[2].data_ptr(), g.shape[1])
        total = int(g.shape[1])
    else:
        t2 = t1
    eng.index_finalize()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    return IngestStats(len(mine), len(mine) * n / eng.sample_rate, n_local, total, t1 - t0 - t_init, t2 - t1,
                       t3 - t2, exchange if world > 1 else "none", t_init, t_synth)
