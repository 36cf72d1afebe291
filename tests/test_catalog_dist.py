"""The N>1 catalog exchange protocol (aidfp.catalog.exchange_postings) under the gloo backend on
CPU, world_size 2 and 3: counts first, one max-padded all-gather, splice in rank order, an empty
rank, u32 bit patterns carried through int32 tensors, postings before `first` kept.

The engine steps it drives (aid_index_shard_info / aid_index_pack / aid_index_splice) are stood in
for by `HostEngine`, a numpy model of their contract (include/aidfp.h); the real ones run the same
protocol on the GPU in tests/test_gpu_comm.py (two ranks on one GPU over gloo) and inside
aid_index_allgather over RCCL (bench.py --gpus N, bench_catalog.py)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aidfp.catalog import exchange_postings, shard


class HostEngine:
    """numpy model of the exchange's three C ABI steps on a host posting store [n, 3]."""

    def __init__(self, post: np.ndarray, n_tracks: int, fail_pack: bool = False):
        self.post = post.astype(np.uint32)
        self.n_tracks = n_tracks
        self._bufs = {}
        self.fail_pack = fail_pack  # aid_engine_force(EXCHANGE_FAIL) stand-in: the pack fails as an OOM would
        self.reserved = None

    def alloc_planes(self, k):
        t = torch.zeros(max(k, 1), dtype=torch.int32)
        self._bufs[t.data_ptr()] = t
        return t[:k] if k else t[:0]

    def _view(self, ptr):
        for base, t in self._bufs.items():
            if base <= ptr < base + 4 * t.numel():
                return t.numpy().view(np.uint32)[(ptr - base) // 4:]
        raise AssertionError("unknown buffer")

    def index_shard_info(self, first):
        return len(self.post) - first, self.n_tracks

    def index_reserve(self, first, total, n_tracks):
        self.reserved = (first, total, n_tracks)  # capacity only: the store itself does not change

    def index_pack(self, first, ptr, stride):
        if self.fail_pack:
            raise MemoryError("injected pack failure")
        v = self._view(ptr)
        n = len(self.post) - first
        assert n <= stride
        for q in range(3):
            v[q * stride: q * stride + n] = self.post[first:, q]
            v[q * stride + n: (q + 1) * stride] = 0

    def index_checksum(self, first=0, count=None):  # aid_index_checksum stand-in: its host mirror
        from aidfp.catalog import checksum_np

        return checksum_np(self.post[first:] if count is None else self.post[first:first + count])

    def index_stats(self):
        return {"postings": len(self.post), "live": len(self.post), "tracks": self.n_tracks}

    def index_splice(self, first, ptr, counts, stride, n_tracks):
        parts = [self.post[:first]]
        if stride:
            v = self._view(ptr)
            for r, n in enumerate(counts):
                blk = v[r * 3 * stride: (r + 1) * 3 * stride].reshape(3, stride)
                parts.append(blk[:, :n].T)
        self.post = np.concatenate(parts, axis=0).astype(np.uint32)
        self.n_tracks = max(self.n_tracks, n_tracks)
        return len(self.post)


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
        b[:, 1] = 100 * r + np.arange(n)  # track column: rank-owned ids
        out.append(b)
    return out


KEEP = np.array([[1, 2, 3], [4, 5, 6]], np.uint32)  # postings before `first`, identical on every rank


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _blocks(world)[rank]
        eng = HostEngine(np.concatenate([KEEP, mine]), n_tracks=100 * rank + len(mine))
        total = exchange_postings(eng, first=len(KEEP))
        q.put((rank, total, eng.post, eng.n_tracks))
    finally:
        dist.destroy_process_group()


def _fail_worker(rank, world, port, q, bad_rank):
    """A world whose rank `bad_rank` fails its pack: every rank must raise (no rank left blocked in the
    payload all-gather) and every index must be unchanged."""
    import time

    from aidfp.catalog import ExchangeAborted

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _blocks(world)[rank]
        start = np.concatenate([KEEP, mine])
        eng = HostEngine(start, n_tracks=100 * rank + len(mine), fail_pack=rank == bad_rank)
        t = time.monotonic()
        kind = "none"
        try:
            exchange_postings(eng, first=len(KEEP))
        except ExchangeAborted:
            kind = "aborted"
        except MemoryError:
            kind = "own"
        # the group is still usable afterwards: the collectives stayed matched
        after = exchange_postings(HostEngine(start, n_tracks=1), first=len(KEEP))
        q.put((rank, kind, time.monotonic() - t, np.array_equal(eng.post, start), after))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bad", [(2, 1), (3, 0)])
def test_exchange_rank_failure_raises_everywhere(world, bad):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, q, bad)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    n_union = len(KEEP) + sum(len(b) for b in _blocks(world))
    for r in range(world):
        kind, dt, unchanged, after = res[r]
        assert kind == ("own" if r == bad else "aborted")
        assert dt < 60 and unchanged
        assert after == n_union


def _agreed_worker(rank, world, port, q):
    from aidfp.catalog import ExchangeAborted, agreed

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def step():
            if rank == 1:
                raise ValueError("rank-local failure")
            return rank

        try:
            agreed(step, "leg")
            kind = "none"
        except ExchangeAborted:
            kind = "aborted"
        except ValueError:
            kind = "own"
        ok = agreed(lambda: rank, "next leg")  # still in step with each other
        q.put((rank, kind, ok))
    finally:
        dist.destroy_process_group()


def test_agreed_leg_failure_reaches_every_rank():
    """bench.py's per-leg agreement: rank 1's exception is raised on rank 1 and ExchangeAborted on the others,
    and the next collective still lines up."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_agreed_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    try:
        res = {r: (k, ok) for r, k, ok in (q.get(timeout=120) for _ in range(3))}
    finally:
        for p in procs:
            p.join(timeout=60)
    assert res == {0: ("aborted", 0), 1: ("own", 1), 2: ("aborted", 2)}


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_postings_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (t, post, nt) for r, t, post, nt in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.concatenate([KEEP] + _blocks(world), axis=0)
    nt_max = max(100 * r + len(b) for r, b in enumerate(_blocks(world)))
    for r in range(world):
        total, post, nt = res[r]
        assert total == len(expect)
        assert np.array_equal(post, expect)
        assert nt == nt_max


def test_shard_balanced_and_complete():
    tracks = np.arange(100003)
    for world in (1, 2, 3, 8):
        parts = [shard(tracks, r, world) for r in range(world)]
        assert np.array_equal(np.concatenate(parts), tracks)
        assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _replica_worker(rank, world, port, q, corrupt_rank):
    """Exchange, then the replica check every bench line carries (catalog.replicas_identical): equal everywhere,
    unless one rank's replica is altered after the exchange."""
    from aidfp.catalog import replica_check

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = _blocks(world)[rank]
        eng = HostEngine(np.concatenate([KEEP, mine]), n_tracks=100 * rank + len(mine))
        exchange_postings(eng, first=len(KEEP))
        if rank == corrupt_rank:
            eng.post = eng.post.copy()
            eng.post[[2, 3]] = eng.post[[3, 2]]  # same postings, two swapped: order matters
        q.put((rank, replica_check(eng)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt", [(2, -1), (3, -1), (3, 2)])
def test_replica_check_gloo(world, corrupt):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_replica_worker, args=(r, world, port, q, corrupt)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = dict(q.get(timeout=120) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in range(world):
        assert res[r]["ranks"] == world
        assert res[r]["replicas_identical"] == (corrupt < 0)
        assert res[r]["mismatched_ranks"] == ([] if corrupt < 0 else [corrupt])


def test_checksum_mirror_properties():
    """aid_index_checksum's host mirror: order-sensitive, position-relative, sensitive to every column."""
    from aidfp.catalog import checksum_np

    rng = np.random.default_rng(1)
    p = rng.integers(0, 2**32, size=(1000, 3), dtype=np.uint64).astype(np.uint32)
    c = checksum_np(p)
    assert c == checksum_np(p.copy()) and 0 <= c < 2**64
    assert checksum_np(p[::-1]) != c
    for col in range(3):
        q = p.copy()
        q[500, col] ^= 1
        assert checksum_np(q) != c
    # a range's checksum counts positions from its own start
    assert checksum_np(p[10:]) == checksum_np(p[10:], 0) != checksum_np(p[10:], 10)
    assert checksum_np(np.zeros((0, 3), np.uint32)) == 0
