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
padding is dropped on receive. The exchange is three engine steps around two
collectives -- aid_index_shard_info, aid_index_pack (shard -> padded device
planes), aid_index_splice (gathered planes -> the index, failure-atomic) -- and
two drivers run them:
  * "native" (default on GPUs): aid_index_allgather in libaidfp runs both
    all-gathers itself over an RCCL communicator the engine owns
    (aid_comm_create; rank 0's unique id is shared with broadcast_object_list)
    -- device postings never leave the C ABI;
  * "torch": `exchange_postings` runs the same pack/splice around
    torch.distributed collectives: RCCL on device tensors ("nccl"), or gloo on
    host copies (several ranks sharing one GPU, tests/test_gpu_comm.py).
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


class ExchangeAborted(RuntimeError):
    """Raised on every rank when some rank could not take part in a collective step (its own error is
    raised on that rank); no rank's index changed."""


def agree(ok: bool, group=None) -> tuple[bool, int]:
    """Collective: every rank learns whether all ranks are ok. Returns (all_ok, first failing rank or -1).
    One all-gather of one int per rank (RCCL on a device tensor under "nccl", else gloo on the host)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return ok, (-1 if ok else 0)
    world = dist.get_world_size(group)
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    mine = torch.tensor([1 if ok else 0], dtype=torch.int64, device=dev)
    allf = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allf, mine, group=group)
    flags = allf.cpu().tolist()
    bad = [r for r, f in enumerate(flags) if not f]
    return not bad, (bad[0] if bad else -1)


def agreed(fn, what: str, group=None):
    """Run the rank-local step `fn()`, then agree on it across the ranks before any later collective: a
    failure on one rank raises on EVERY rank (its own exception there, ExchangeAborted elsewhere) instead
    of leaving the others blocked in the next collective."""
    err = None
    out = None
    try:
        out = fn()
    except Exception as exc:  # noqa: BLE001 - re-raised below on this rank
        err = exc
    ok, bad = agree(err is None, group)
    if err is not None:
        raise err
    if not ok:
        raise ExchangeAborted(f"{what}: rank {bad} failed; aborted on every rank")
    return out


def exchange_postings(eng, first: int = 0, group=None) -> int:
    """Replace this rank's postings [first, n) by the union of every rank's, in rank order, through
    torch.distributed collectives around aid_index_reserve / aid_index_pack / aid_index_splice. Returns
    the postings held.

    Every rank runs the same collectives whatever happens locally: the (count, n_tracks) all-gather, then
    one ok flag after the local preparation (exchange buffers, the grown index, the pack), and the payload
    only if every rank is ready -- a rank-local failure raises on every rank with the indexes unchanged
    (native twin: aid_index_allgather). Under "nccl" the planes are all-gathered as device tensors; under
    gloo as host copies. `eng` needs index_shard_info / index_pack / index_splice (index_reserve when it
    has one) and device buffers from `eng.alloc_planes` when it has one (tests use a host stand-in), else
    torch.cuda tensors."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    on_dev = dist.get_backend(group) == "nccl"
    err = None
    try:
        n, nt = eng.index_shard_info(first)
    except Exception as exc:  # noqa: BLE001 - still takes part in the counts round (count -1)
        err, n, nt = exc, -1, 0
    meta = torch.tensor([n, nt], dtype=torch.int64, device="cuda" if on_dev else "cpu")
    allm = torch.empty(2 * world, dtype=torch.int64, device=meta.device)
    dist.all_gather_into_tensor(allm, meta, group=group)
    m = allm.view(world, 2).cpu().numpy()
    if err is not None:
        raise err
    if (m[:, 0] < 0).any():
        raise ExchangeAborted(f"index exchange: rank {int(np.argmax(m[:, 0] < 0))} has an invalid shard")
    counts, stride, tracks = m[:, 0].copy(), int(m[:, 0].max()), int(m[:, 1].max())
    alloc = getattr(eng, "alloc_planes", None) or (lambda k: torch.empty(k, dtype=torch.int32, device="cuda"))

    def prepare():
        send = alloc(3 * stride)
        recv = alloc(3 * stride * world)
        reserve = getattr(eng, "index_reserve", None)
        if reserve is not None:
            reserve(first, int(counts.sum()), tracks)
        if stride:
            eng.index_pack(first, send.data_ptr(), stride)
        return send, recv

    send, recv = agreed(prepare, "index exchange (prepare)", group)
    if on_dev:
        if stride:
            dist.all_gather_into_tensor(recv, send, group=group)
        torch.cuda.synchronize()  # the engine's stream reads what torch's stream gathered
    else:
        recv_h = torch.empty(3 * stride * world, dtype=torch.int32)
        if stride:
            dist.all_gather_into_tensor(recv_h, send.cpu(), group=group)
        recv.copy_(recv_h)
    return eng.index_splice(first, recv.data_ptr() if stride else 0, counts, stride, tracks)


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def checksum_np(postings: np.ndarray, first_index: int = 0) -> int:
    """Host mirror of aid_index_checksum over a [n, 3] uint32 (hash, track, t) array whose row 0 sits at position
    `first_index` of the checksummed range (tests; the replicas are checksummed on the device)."""
    p = np.asarray(postings, dtype=np.uint32).reshape(-1, 3).astype(np.uint64)
    i = np.arange(first_index, first_index + len(p), dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = ((p[:, 0] << np.uint64(32)) | p[:, 2]) ^ (p[:, 1] * np.uint64(0x9E3779B97F4A7C15)) ^ \
            (i * np.uint64(0xD6E8FEB86659FD93))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        return int(np.add.reduce(z, dtype=np.uint64)) if len(z) else 0


def replica_check(eng, group=None) -> dict:
    """Collective: every rank checksums its whole replica on the device (aid_index_checksum) and the checksums
    are all-gathered; `replicas_identical` is true when every rank holds the same postings in the same order."""
    import torch.distributed as dist

    def local():
        return eng.index_checksum(), eng.index_stats()["postings"]

    if dist.is_available() and dist.is_initialized():
        mine, n = agreed(local, "replica checksum", group)  # a rank that cannot checksum fails every rank
        allc = [None] * dist.get_world_size(group)
        dist.all_gather_object(allc, (mine, n), group=group)
    else:
        mine, n = local()
        allc = [(mine, n)]
    return {"replicas_identical": len({c for c, _ in allc}) == 1 and len({k for _, k in allc}) == 1,
            "checksum": f"{mine:016x}", "ranks": len(allc),
            "mismatched_ranks": [r for r, (c, k) in enumerate(allc) if (c, k) != allc[0]]}


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
    rccl_nranks: int = 0  # ranks of the native RCCL communicator (ncclCommCount), 0 = none used


def native_comm(eng, group=None) -> int:
    """aid_comm over the ranks of `group`: rank 0's RCCL id is broadcast through torch.distributed."""
    import torch.distributed as dist

    rank = dist.get_rank(group)
    obj = [agreed(lambda: eng.comm_id() if rank == 0 else None, "RCCL unique id", group)]
    dist.broadcast_object_list(obj, src=0, group=group)
    return eng.comm_create(obj[0], dist.get_world_size(group), rank)


def ingest_synthetic(eng, track_ids, seconds: float, batch: int = 256, group=None,
                     exchange: str = "native", source_sr: int | None = None, local: bool = False) -> IngestStats:
    """Fingerprint this rank's shard of synthetic tracks on its GPU, replicate the index.

    `track_ids` is the full catalog (global ids); with torch.distributed initialised (and `local` False)
    each rank takes shard(track_ids, rank, world), otherwise the whole list. `source_sr`: the tracks are
    synthesised at that rate and brought to the engine's rate by K6 per track, as ingest decodes every file
    with ffmpeg `-ar 16000` (audio-ident-service/app/audio/decode.py:41-60); default: synthesised at the
    engine's rate."""
    import torch
    import torch.distributed as dist

    distributed = dist.is_available() and dist.is_initialized() and not local
    rank = dist.get_rank(group) if distributed else 0
    world = dist.get_world_size(group) if distributed else 1
    mine = np.asarray(shard(np.asarray(track_ids, dtype=np.uint32), rank, world), dtype=np.uint32)
    resample = source_sr is not None and int(source_sr) != eng.sample_rate
    if resample:
        n_src = int(round(seconds * source_sr)) & ~1
        n = eng.resample_len(n_src, int(source_sr), eng.sample_rate) & ~1
    else:
        n = int(round(seconds * eng.sample_rate)) & ~1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    base = eng.index_stats()["postings"]
    ev = []

    def extract_shard():
        nb = max(1, min(batch, len(mine)))
        pcm = torch.empty(nb * n, dtype=torch.float32, device="cuda")
        src = torch.empty(nb * n_src, dtype=torch.float32, device="cuda") if resample else None
        # one non-default stream for generation, extraction and the posting append: events recorded on
        # the legacy default stream would serialise against the engine's (blocking) stream every batch.
        # Nothing in the loop waits for its own batch (the generation is enqueued, the append scans its
        # counts on the device): the host runs ahead and the GPU goes from batch to batch without a gap
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        for b0 in range(0, len(mine), batch):
            tr = mine[b0 : b0 + batch]
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            if resample:  # each track decoded at its own rate, then K6 to the engine's (ffmpeg -ar per file)
                eng.synth(src.data_ptr(), tr, np.zeros(len(tr), np.int64), n_src, stream=s.cuda_stream,
                          sample_rate=int(source_sr), wait=False)
                for c in range(len(tr)):
                    eng.resample_range(src.data_ptr() + 4 * c * n_src, 0, n_src, 1, int(source_sr), eng.sample_rate,
                                       0, n, pcm.data_ptr() + 4 * c * n, stream=s.cuda_stream)
            else:
                eng.synth(pcm.data_ptr(), tr, np.zeros(len(tr), np.int64), n, stream=s.cuda_stream, wait=False)
            b.record(s)
            ev.append((a, b))
            eng.extract_device(pcm.data_ptr(), np.arange(len(tr) + 1, dtype=np.int64) * n, s.cuda_stream)
            eng.index_add_extracted(tr)
        del pcm, src
        torch.cuda.synchronize()

    if distributed and world > 1:
        agreed(extract_shard, "catalog ingest (extract)", group)  # a failed shard stops every rank here
    else:
        extract_shard()
    t1 = time.perf_counter()
    t_synth = sum(a.elapsed_time(b) for a, b in ev) * 1e-3
    n_local = eng.index_stats()["postings"] - base
    total = n_local
    t_init = 0.0
    nranks = 0
    if world > 1 and exchange == "native":
        ti = time.perf_counter()
        comm = native_comm(eng, group)  # collective; aid_index_allgather agrees on every rank's readiness itself
        t1 = time.perf_counter()
        t_init = t1 - ti
        try:
            nranks = eng.comm_size(comm)[0]
            total = eng.index_allgather(comm, base) - base
        finally:
            eng.comm_destroy(comm)
        t2 = time.perf_counter()
    elif world > 1:
        total = exchange_postings(eng, base, group) - base
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    else:
        t2 = t1
    eng.index_finalize()
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    return IngestStats(len(mine), len(mine) * n / eng.sample_rate, n_local, total, t1 - t0 - t_init, t2 - t1,
                       t3 - t2, exchange if world > 1 else "none", t_init, t_synth, nranks)
