"""GPU: the native exchange (aid_comm_* + aid_index_allgather) through the C ABI.

A one-GPU box only allows a world-1 RCCL communicator (RCCL refuses two ranks on one
device), so this pins the plumbing and the bookkeeping: the gathered union of a single
rank is its own shard in order, postings before `first` stay, the track tables grow, and
the finalized index answers queries exactly as before the exchange. The multi-rank data
movement is the same padded-all-gather scheme that tests/test_catalog_dist.py checks
under gloo (counts first, pad to max, drop the padding in rank order).
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
