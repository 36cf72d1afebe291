"""The N>1 catalog exchange (aidfp.catalog.allgather_postings) under the gloo
backend on CPU, world_size 2 and 3: variable counts, an empty rank, rank-order
concatenation, u32 bit patterns carried through int32 tensors. The GPU path runs
the same function over RCCL (bench_catalog.py)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aidfp.catalog import allgather_postings, shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _blocks(world):
    rng = np.random.default_rng(0)
    sizes = [5, 0, 17][:world] if world == 3 else [3, 11]
    out = []
    for r, n in enumerate(sizes):
        b = rng.integers(0, 2**32, size=(n, 3), dtype=np.uint64).astype(np.uint32)
        b[:, 1] = r  # track column encodes the rank
        out.append(b)
    return out


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = torch.from_numpy(_blocks(world)[rank].astype(np.int32))
        got = allgather_postings(mine)
        q.put((rank, got.numpy().astype(np.uint32)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allgather_postings_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.concatenate(_blocks(world), axis=0)
    for r in range(world):
        assert np.array_equal(res[r], expect)


def test_shard_balanced_and_complete():
    tracks = np.arange(100003)
    for world in (1, 2, 3, 8):
        parts = [shard(tracks, r, world) for r in range(world)]
        assert np.array_equal(np.concatenate(parts), tracks)
        assert max(map(len, parts)) - min(map(len, parts)) <= 1
