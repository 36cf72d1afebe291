"""GPU: the native exchange (aid_comm_* + aid_index_allgather) through the C ABI.

A one-GPU box only allows a world-1 RCCL communicator (RCCL refuses two ranks on one
device): the world-1 test pins the native plumbing (the gathered union of a single rank is its
own shard in order, postings before `first` stay, the track tables grow, the finalized index
answers queries exactly as before). The multi-rank data movement runs the same engine steps
(aid_index_pack -> all-gather -> aid_index_splice) with two real ranks sharing the GPU over gloo
(test_world2_exchange_on_one_gpu); the 8-GPU RCCL run is bench.py --gpus 8's catalog leg.
"""

import numpy as np
import pytest

from aidfp import synth

pytestmark = pytest.mark.gpu
SR = 44100


def test_allgather_world1_keeps_index(gpu_engine):
    import oracle as O

    eng = gpu_engine
    eng.index_reset()
    ids_a, ids_b = [100, 101], [0, 1, 2, 3]
    eng.extract_host([synth.synth(t, 0, SR * 8, SR, salt=5) for t in ids_a])
    eng.index_add_extracted(np.array(ids_a, np.uint32))
    first = eng.index_stats()["postings"]
    eng.extract_host([synth.synth(t, 0, SR * 8, SR, salt=5) for t in ids_b])
    eng.index_add_extracted(np.array(ids_b, np.uint32))
    before = eng.index_export()
    comm = eng.comm_create(eng.comm_id(), 1, 0)
    try:
        assert eng.comm_size(comm) == (1, 0)
        n = eng.index_allgather(comm, first)
        assert n == len(before)
        assert np.array_equal(eng.index_export(), before)
        n0 = eng.index_allgather(comm, 0)  # whole index as the shard
        assert n0 == len(before)
        assert np.array_equal(eng.index_export(), before)
    finally:
        eng.comm_destroy(comm)
    eng.index_finalize()
    qt = [1, 101, 3, 77]  # 77 is not indexed
    q = [synth.synth(t, SR, SR * 5, SR, snr_db=20.0, salt=9) for t in qt]
    got = eng.extract_host(q)
    rows = eng.query_extracted()
    for t, r, rec in zip(qt, rows, got):
        ref = O.query(before, rec, min_match=eng.min_match, max_rows=eng.max_results)
        assert np.array_equal(r, ref), f"query {t}"
    assert [int(r[0, 1]) if len(r) else None for r in rows] == [1, 101, 3, None]


def test_allgather_bad_arguments(gpu_engine):
    from aidfp._lib import EngineError

    comm = gpu_engine.comm_create(gpu_engine.comm_id(), 1, 0)
    try:
        n = gpu_engine.index_stats()["postings"]
        with pytest.raises(EngineError):
            gpu_engine.index_allgather(comm, n + 1)
    finally:
        gpu_engine.comm_destroy(comm)
    with pytest.raises(ValueError):
        gpu_engine.comm_create(b"short", 1, 0)


def test_allgather_injected_failure_world1(gpu_engine):
    """aid_index_allgather's ok round: a failure of this rank's prepare step (injected through
    aid_engine_force EXCHANGE_FAIL) returns an error after the agreement, the index is unchanged, and the
    next exchange over the same communicator works (the collectives stayed matched)."""
    from aidfp._lib import EngineError

    eng = gpu_engine
    eng.index_reset()
    eng.extract_host([synth.synth(t, 0, SR * 6, SR, salt=5) for t in (1, 2, 3)])
    eng.index_add_extracted(np.array([1, 2, 3], np.uint32))
    before = eng.index_export()
    comm = eng.comm_create(eng.comm_id(), 1, 0)
    try:
        eng.force("exchange_fail", 1)
        with pytest.raises(EngineError, match="injected"):
            eng.index_allgather(comm, 0)
        assert np.array_equal(eng.index_export(), before)
        assert eng.index_stats()["tracks"] == 4
        assert eng.index_allgather(comm, 0) == len(before)  # the hook is one-shot
        assert np.array_equal(eng.index_export(), before)
    finally:
        eng.comm_destroy(comm)


def test_splice_failure_leaves_index(gpu_engine):
    """aid_index_splice validates before it touches the index: a bad count fails and nothing changes."""
    import torch

    from aidfp._lib import EngineError

    eng = gpu_engine
    eng.index_reset()
    eng.extract_host([synth.synth(t, 0, SR * 6, SR, salt=5) for t in (3, 4)])
    eng.index_add_extracted(np.array([3, 4], np.uint32))
    before = eng.index_export()
    recv = torch.zeros(3 * 8, dtype=torch.int32, device="cuda")
    with pytest.raises(EngineError):
        eng.index_splice(0, recv.data_ptr(), [9], 8, 10)  # count 9 > stride 8
    assert np.array_equal(eng.index_export(), before)
    assert eng.index_stats()["tracks"] == 5


def _rank_worker(rank, world, port, q):
    """One rank of a world-2 catalog on ONE GPU: real engines, pack/splice through the C ABI, gloo
    moving host copies of the padded planes (RCCL refuses two ranks on one device)."""
    import os

    import torch.distributed as dist

    from aidfp.catalog import exchange_postings
    from aidfp.engine import Engine

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with Engine(SR, device=0) as eng:
            ids = [10 * rank + k for k in range(2 + rank)]  # 2 and 3 tracks: unequal shards (padding)
            eng.extract_host([synth.synth(t, 0, SR * 9, SR, salt=5) for t in ids])
            eng.index_add_extracted(np.array(ids, np.uint32))
            mine = eng.index_export()
            total = exchange_postings(eng, 0)
            union = eng.index_export()
            eng.index_finalize()
            qt = [1, 11, 12, 99]
            qs = [synth.synth(t, SR, SR * 5, SR, snr_db=20.0, salt=9) for t in qt]
            recs = eng.extract_host(qs)
            rows = eng.query_extracted()
            q.put((rank, mine, total, union, eng.index_stats()["tracks"], recs, rows))
    finally:
        dist.destroy_process_group()


def _fail_rank_worker(rank, world, port, q):
    """World 2 on one GPU, rank 1's pack fails by injection: both ranks must raise, indexes unchanged."""
    import os
    import time

    import torch.distributed as dist

    from aidfp._lib import EngineError
    from aidfp.catalog import ExchangeAborted, exchange_postings
    from aidfp.engine import Engine

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        with Engine(SR, device=0) as eng:
            ids = [10 * rank + k for k in range(2 + rank)]
            eng.extract_host([synth.synth(t, 0, SR * 6, SR, salt=5) for t in ids])
            eng.index_add_extracted(np.array(ids, np.uint32))
            mine = eng.index_export()
            tracks = eng.index_stats()["tracks"]
            if rank == 1:
                eng.force("exchange_fail", 1)
            t = time.monotonic()
            kind = "none"
            try:
                exchange_postings(eng, 0)
            except EngineError as exc:
                kind = "own:" + str(exc)[:80]
            except ExchangeAborted:
                kind = "aborted"
            dt = time.monotonic() - t
            same = np.array_equal(eng.index_export(), mine) and eng.index_stats()["tracks"] == tracks
            total = exchange_postings(eng, 0)  # the retry succeeds on both ranks
            q.put((rank, kind, dt, same, total))
    finally:
        dist.destroy_process_group()


def test_world2_rank_failure_on_one_gpu():
    """The N-rank exchange's failure agreement with real engines: rank 1's pack fails (aid_engine_force
    EXCHANGE_FAIL), rank 1 raises its own EngineError, rank 0 raises ExchangeAborted -- both within seconds,
    neither blocked in the payload all-gather -- and both indexes are unchanged; a retry then succeeds."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fail_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            item = q.get(timeout=300)
            res[item[0]] = item[1:]
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    assert res[0][0] == "aborted"
    assert res[1][0].startswith("own:") and "injected" in res[1][0]
    for r in (0, 1):
        _, dt, same, total = res[r]
        assert dt < 60 and same
    assert res[0][3] == res[1][3] > 0


def test_world2_exchange_on_one_gpu():
    """Two processes, one GPU, gloo: each rank's index after the exchange is the concatenation of the
    shards in rank order (rank 0's 2 tracks, then rank 1's 3), and queries against it equal the
    oracle's rows over that union."""
    import socket

    import torch.multiprocessing as mp

    import oracle as O

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            item = q.get(timeout=300)
            res[item[0]] = item[1:]
    finally:
        for p in procs:
            p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    expect = np.concatenate([res[0][0], res[1][0]], axis=0)
    assert len(res[0][0]) > 0 and len(res[1][0]) > len(res[0][0])
    for r in (0, 1):
        _, total, union, n_tracks, recs, rows = res[r]
        assert total == len(expect)
        assert np.array_equal(union, expect)
        assert n_tracks == 13
        for rec, row in zip(recs, rows):
            ref = O.query(union, rec, min_match=10, max_rows=50)  # the FPSPEC v1 default of the ranks' engines
            assert np.array_equal(row, ref)
        assert [int(x[0, 1]) if len(x) else None for x in rows] == [1, 11, 12, None]
