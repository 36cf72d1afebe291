"""K5 under heavy vote load (popular hashes, as a 100k-track catalog has them): rows stay
identical to the CPU oracle (oracle/fp_match.c, FPSPEC 7) on the LDS fast path (forced, up to
~10 votes per 16-bit counter; overflows fall back), on the global-histogram path (forced) and
on the engine's own choice. "global2" splits K5a's keys over two workgroups per query (the
engine's choice above 2^18 votes)."""

import numpy as np
import pytest

import oracle as O
from aidfp import synth
from aidfp.engine import Engine

pytestmark = pytest.mark.gpu
SR = 44100
HOP = 512


@pytest.mark.parametrize("path", ["auto", "lds", "global", "global2"])
@pytest.mark.parametrize("per_hash", [0, 30, 90, 160])
def test_rows_equal_oracle_under_load(per_hash, path):
    rng = np.random.default_rng(per_hash)
    track = synth.synth(7, 0, 30 * SR, SR)
    trec = O.fingerprint(track, HOP)
    queries = [synth.synth(7, s, 5 * SR, SR, snr_db=20.0, salt=3 + i) for i, s in enumerate((SR * 4, SR * 17))]
    qrecs = [O.fingerprint(q, HOP) for q in queries]
    h = [(trec & np.uint64(0xFFFFFFFF)).astype(np.uint32)]
    tr = [np.full(len(trec), 7, np.uint32)]
    t = [(trec >> np.uint64(32)).astype(np.uint32)]
    if per_hash:
        # per_hash postings of random tracks/times for every distinct query hash: chance votes
        qh = np.unique(np.concatenate([(r & np.uint64(0xFFFFFFFF)).astype(np.uint32) for r in qrecs]))
        h.append(np.repeat(qh, per_hash))
        tr.append(rng.integers(1000, 9000, len(qh) * per_hash).astype(np.uint32))
        t.append(rng.integers(0, 3000, len(qh) * per_hash).astype(np.uint32))
        # and a few tracks that share a block of the query's hashes at one offset (near-duplicates)
        for k in range(6):
            sel = qrecs[0][rng.permutation(len(qrecs[0]))[: 15 + 7 * k]]
            h.append((sel & np.uint64(0xFFFFFFFF)).astype(np.uint32))
            tr.append(np.full(len(sel), 20000 + k, np.uint32))
            t.append(((sel >> np.uint64(32)) + np.uint64(100 + k)).astype(np.uint32))
    H, TR, T = (np.ascontiguousarray(np.concatenate(a)) for a in (h, tr, t))
    with Engine(SR) as eng:
        eng.force("k5_path", {"auto": 0, "lds": 1, "global": 2, "global2": 2}[path])
        eng.force("k5_parts", 2 if path == "global2" else 0)
        eng.index_add_postings(H.ctypes.data, TR.ctypes.data, T.ctypes.data, len(H), device=False)
        eng.index_finalize()
        post = eng.index_export()
        got = eng.query(qrecs)
        for g, r in zip(got, qrecs):
            ref = O.query(post, r, min_match=eng.min_match, max_rows=eng.max_results)
            assert np.array_equal(g, ref), (per_hash, g[:4], ref[:4])
            assert len(g) and g[0, 1] == 7


def test_mixed_batch_routes_each_query_by_its_votes():
    """in one batch, queries above the LDS filter's bound (2^18 votes) go straight to the global path
    while the light ones are answered in LDS; rows equal the oracle's either way."""
    rng = np.random.default_rng(11)
    track = synth.synth(7, 0, 30 * SR, SR)
    trec = O.fingerprint(track, HOP)
    q = synth.synth(7, SR * 9, 5 * SR, SR, snr_db=20.0, salt=5)
    qrec = O.fingerprint(q, HOP)
    qh = np.unique((qrec & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    per_hash = 600
    H = np.ascontiguousarray(np.concatenate([(trec & np.uint64(0xFFFFFFFF)).astype(np.uint32), np.repeat(qh, per_hash)]))
    TR = np.ascontiguousarray(np.concatenate([np.full(len(trec), 7, np.uint32),
                                              rng.integers(1000, 9000, len(qh) * per_hash).astype(np.uint32)]))
    T = np.ascontiguousarray(np.concatenate([(trec >> np.uint64(32)).astype(np.uint32),
                                             rng.integers(0, 3000, len(qh) * per_hash).astype(np.uint32)]))
    heavy = [qrec, qrec[::-1].copy()]
    light = [qrec[:60], qrec[200:260]]
    with Engine(SR) as eng:
        eng.index_add_postings(H.ctypes.data, TR.ctypes.data, T.ctypes.data, len(H), device=False)
        eng.index_finalize()
        post = eng.index_export()
        qs = [heavy[0], light[0], heavy[1], light[1]] + [qrec[i:i + 40] for i in range(0, 600, 40)]
        eng.match_stats(reset=True)
        got = eng.query(qs)
        st = eng.match_stats(reset=True)
        for g, r in zip(got, qs):
            assert np.array_equal(g, O.query(post, r, min_match=eng.min_match, max_rows=eng.max_results))
        votes_heavy = len(qrec) * per_hash
        assert votes_heavy > (1 << 18)
        assert st["queries_global"] == 2 and st["queries_lds"] == len(qs) - 2, st


def test_lds_path_keeps_four_workgroups_per_cu():
    """k_match_lds is laid out for exactly 40 KB of LDS (FPSPEC v1's distinct-frame set included): four resident
    workgroups per CU, the occupancy its timing was tuned at."""
    from aidfp.engine import Engine

    with Engine(44100) as eng:
        assert eng.match_stats()["lds_path_workgroups_per_cu"] == 4
