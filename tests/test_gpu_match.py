"""GPU parity for K4 index build + K5 match_vote vs the CPU oracle (oracle/fp_match.c,
FPSPEC 7), plus the identification behaviour the reference's exact lane relies on
(audio-ident-service/app/search/exact.py: best track first, offset recovered)."""

import numpy as np
import pytest

import oracle as O
from aidfp import synth
from aidfp.engine import Engine

pytestmark = pytest.mark.gpu
SR = 44100
HOP = 512
N_TRACKS = 48
TRACK_S = 30


@pytest.fixture(scope="module")
def catalog():
    import torch

    eng = Engine(SR)
    n = SR * TRACK_S
    pcm = torch.empty(N_TRACKS * n, dtype=torch.float32, device="cuda")
    tracks = np.arange(N_TRACKS, dtype=np.uint32) + 500
    eng.synth(pcm.data_ptr(), tracks, np.zeros(N_TRACKS, np.int64), n)
    eng.extract_device(pcm.data_ptr(), np.arange(N_TRACKS + 1, dtype=np.int64) * n)
    eng.index_add_extracted(tracks)
    eng.index_finalize()
    yield eng, tracks
    eng.close()


def _queries(tracks, rng, n_q=12, neg=3):
    qs, truth = [], []
    for i in range(n_q):
        tr = int(tracks[rng.integers(len(tracks))])
        start = int(rng.integers(0, (TRACK_S - 5) * SR))
        qs.append(synth.synth(tr, start, 5 * SR, SR, snr_db=20.0, salt=100 + i))
        truth.append((tr, start))
    for i in range(neg):  # unseen tracks
        qs.append(synth.synth(90000 + i, 0, 5 * SR, SR, snr_db=20.0, salt=7))
        truth.append((None, 0))
    return qs, truth


def test_match_rows_equal_oracle(catalog):
    eng, tracks = catalog
    st = eng.index_stats()
    post = eng.index_export()
    assert st["postings"] == len(post) == st["live"] > 0
    rng = np.random.default_rng(42)
    qs, truth = _queries(tracks, rng)
    # query records from the GPU extractor are bit-exact to the oracle's (tests/test_gpu_extract.py)
    recs = [O.fingerprint(q, HOP) for q in qs]
    got = eng.query(recs)
    for q, (g, r) in enumerate(zip(got, recs)):
        ref = O.query(post, r, min_match=eng.min_match, max_rows=eng.max_results)
        assert np.array_equal(g, ref), f"query {q}: rows differ\n{g[:5]}\n{ref[:5]}"
    # identification: true track ranked first, offset recovered to within one hop
    for g, (tr, start) in zip(got, truth):
        if tr is None:
            assert len(g) == 0 or g[0, 0] < 20
            continue
        assert g[0, 1] == tr
        assert abs(g[0, 2] * HOP - start) <= HOP


def test_level_and_band_robustness(catalog):
    """FPSPEC 5's peak threshold is absolute, so a query's recording level moves peaks across it. The index holds
    unit-gain tracks; 5 s queries at 0 / -12 / -24 dB (20 dB SNR noise) and a 300-3400 Hz phone band must still
    rank the true track first with its offset (the reference's exact-lane categories, scripts/eval_exact.py:46-54;
    measured at scale in profiles/r03_config4_match.json). Runs before test_remove_and_save_load removes a track
    from the shared catalog."""
    from scipy.signal import butter, sosfilt

    eng, tracks = catalog
    rng = np.random.default_rng(11)
    sos = butter(4, [300.0, 3400.0], btype="bandpass", fs=SR, output="sos")
    qs, truth = [], []
    for i in range(8):
        tr = int(tracks[rng.integers(len(tracks))])
        start = int(rng.integers(0, (TRACK_S - 5) * SR))
        x = synth.synth(tr, start, 5 * SR, SR, snr_db=20.0, salt=300 + i).astype(np.float64)
        for kind in ("0dB", "-12dB", "-24dB", "phone"):
            y = sosfilt(sos, x) if kind == "phone" else x * 10.0 ** (float(kind[:-2]) / 20.0)
            qs.append(y.astype(np.float32))
            truth.append((tr, start, kind))
    got = eng.query_pcm(qs)
    for g, (tr, start, kind) in zip(got, truth):
        assert len(g) > 0 and g[0, 1] == tr, f"{kind}: true track {tr} not first: {g[:3]}"
        assert abs(g[0, 2] * HOP - start) <= HOP, kind

def test_lds_counter_wrap_long_queries(catalog):
    """Clean 25 s excerpts give their (track, d) thousands of votes: the LDS path's 8-bit filter counters wrap many
    times (a wrapped bucket, and each full counter its carry runs through, is marked hot directly). Rows on the LDS
    path and on the global-histogram path must both equal the oracle's."""
    eng, tracks = catalog
    post = eng.index_export()
    qs = [synth.synth(int(tracks[i]), (i + 1) * 7919, 25 * SR, SR) for i in (1, 5, 9)]
    qs.append(np.concatenate([qs[0][: 10 * SR], qs[1][: 10 * SR]]))  # two tracks, each far past 255
    recs = [O.fingerprint(q, HOP) for q in qs]
    refs = [O.query(post, r, min_match=eng.min_match, max_rows=eng.max_results) for r in recs]

    def raw_votes(rec, row):  # the filter counts raw votes; FPSPEC v1's match_count counts distinct anchor frames
        tr, d = int(row[1]), int(row[2])
        p = post[post[:, 1] == tr]
        have = set(zip(p[:, 0].tolist(), p[:, 2].tolist()))
        h, tq = (rec & np.uint64(0xFFFFFFFF)).astype(np.int64), (rec >> np.uint64(32)).astype(np.int64)
        return sum((int(a), int(b) + d) in have for a, b in zip(h, tq))

    assert all(r[0, 0] > 100 for r in refs[:3]) and refs[3][1, 0] > 50
    assert all(raw_votes(recs[i], refs[i][0]) > 1000 for i in range(3)) and raw_votes(recs[3], refs[3][1]) > 255
    try:
        for path in (1, 2):
            eng.force("k5_path", path)
            st0 = eng.match_stats(reset=True)
            got = eng.query(recs)
            st = eng.match_stats(reset=True)
            for q, (g, r) in enumerate(zip(got, refs)):
                assert np.array_equal(g, r), f"path {path} query {q}"
            if path == 1:  # answered in LDS, no fallback to the global path
                assert st["queries_lds"] == len(qs) and st["queries_global"] == 0, (st0, st)
    finally:
        eng.force("k5_path", 0)


def test_query_extracted_equals_host_query(catalog):
    eng, tracks = catalog
    rng = np.random.default_rng(7)
    qs, _ = _queries(tracks, rng, n_q=6, neg=1)
    recs = eng.extract_host(qs)
    dev = eng.query_extracted()
    host = eng.query(recs)
    for a, b in zip(dev, host):
        assert np.array_equal(a, b)


def test_remove_and_save_load(catalog, tmp_path):
    eng, tracks = catalog
    rng = np.random.default_rng(3)
    qs, truth = _queries(tracks, rng, n_q=4, neg=0)
    recs = [O.fingerprint(q, HOP) for q in qs]
    victim = truth[0][0]
    path = tmp_path / "idx.aidfp"
    eng.index_save(str(path))
    eng.index_remove(victim)
    with pytest.raises(Exception):
        eng.index_remove(victim)  # already removed
    post = eng.index_export()
    live = post[post[:, 1] != victim]
    got = eng.query(recs)
    for g, r in zip(got, recs):
        assert victim not in set(g[:, 1].tolist())
        assert np.array_equal(g, O.query(live, r, min_match=eng.min_match, max_rows=eng.max_results))
    # a fresh engine loading the saved file answers like the original did before the removal
    with Engine(SR) as e2:
        e2.index_load(str(path))
        g2 = e2.query(recs)
    for g, r in zip(g2, recs):
        assert np.array_equal(g, O.query(post, r, min_match=eng.min_match, max_rows=eng.max_results))


def test_empty_index_and_empty_query():
    with Engine(16000) as eng:
        eng.index_finalize()
        out = eng.query([np.zeros(0, np.uint64), O.fingerprint(synth.synth(1, 0, 16000 * 4, 16000), 256)])
        assert [len(o) for o in out] == [0, 0]


def _small_catalog(eng, n_tracks=6, seconds=12, sr=16000):
    import torch

    n = sr * seconds
    pcm = torch.empty(n_tracks * n, dtype=torch.float32, device="cuda")
    tracks = np.arange(n_tracks, dtype=np.uint32) + 10
    eng.synth(pcm.data_ptr(), tracks, np.zeros(n_tracks, np.int64), n)
    eng.extract_device(pcm.data_ptr(), np.arange(n_tracks + 1, dtype=np.int64) * n)
    eng.index_add_extracted(tracks)
    torch.cuda.synchronize()
    return tracks


def test_compact_drops_removed_postings_in_order(tmp_path):
    """aid_index_compact (removed tracks' postings were never reclaimed): the stored
    postings become exactly the live ones, in their order, and query rows do not change."""
    sr, hop = 16000, 256
    with Engine(sr) as eng:
        tracks = _small_catalog(eng)
        before = eng.index_export()
        q = [O.fingerprint(synth.synth(int(t), sr * 3, sr * 4, sr, snr_db=20.0, salt=5), hop) for t in tracks[:4]]
        for victim in (tracks[1], tracks[4]):
            eng.index_remove(int(victim))
        rows_before = eng.query(q)
        dropped = eng.index_compact()
        after = eng.index_export()
        keep = ~np.isin(before[:, 1], [tracks[1], tracks[4]])
        assert dropped == int((~keep).sum()) > 0
        assert np.array_equal(after, before[keep])
        rows_after = eng.query(q)
        for a, b, r in zip(rows_before, rows_after, q):
            assert np.array_equal(a, b)
            assert np.array_equal(b, O.query(after, r, min_match=eng.min_match, max_rows=eng.max_results))
        assert eng.index_compact() == 0  # nothing left to drop
        with pytest.raises(Exception):
            eng.index_remove(int(tracks[1]))  # still removed (tombstones survive compaction)


def test_failed_load_leaves_the_index_untouched(tmp_path):
    """aid_index_load validates the file and reads it into scratch buffers first; a
    bad or truncated file fails without changing the loaded index."""
    sr, hop = 16000, 256
    with Engine(sr) as eng:
        _small_catalog(eng, n_tracks=3)
        good = tmp_path / "good.aidfp"
        eng.index_save(str(good))
        post = eng.index_export()
        st = eng.index_stats()
        q = [O.fingerprint(synth.synth(11, sr * 2, sr * 4, sr), hop)]
        rows = eng.query(q)
        blob = good.read_bytes()
        bad = {
            "truncated": blob[: len(blob) - 5],
            "trailing": blob + b"\0",
            "magic": b"XXXXXXXX" + blob[8:],
            "abi": blob[:8] + np.int64(99).tobytes() + blob[16:],
            "negative": blob[:32] + np.int64(-1).tobytes() + blob[40:],
        }
        for what, data in bad.items():
            p = tmp_path / f"{what}.aidfp"
            p.write_bytes(data)
            with pytest.raises(Exception):
                eng.index_load(str(p))
            assert eng.index_stats()["postings"] == st["postings"], what
            assert np.array_equal(eng.index_export(), post), what
            assert all(np.array_equal(a, b) for a, b in zip(eng.query(q), rows)), what
        with Engine(sr) as e2:
            e2.index_load(str(good))
            assert np.array_equal(e2.index_export(), post)


def test_zero_hash_track_has_a_slot():
    """a track with no hashes (shorter than one frame) can be removed after it is added."""
    with Engine(16000) as eng:
        recs = eng.extract_host([np.zeros(1000, np.float32)])[0]
        assert len(recs) == 0
        eng.index_add_records(77, recs)
        assert eng.index_stats()["tracks"] == 78
        eng.index_remove(77)
        with pytest.raises(Exception):
            eng.index_remove(77)


def test_sort_build_equals_atomic_build():
    """K4 hand-written radix-sort build (index_sort.hip, default), its ballot-ranked form (force k4_build 4) and the
    atomic counting sort (force 2): same live postings and identical query rows, with removed tracks (sentinel keys
    sorted past the live ones)."""
    import torch

    n = SR * 12
    tracks = np.arange(20, dtype=np.uint32) * 7 + 3
    rng = np.random.default_rng(5)
    qs = [synth.synth(int(tracks[i]), int(rng.integers(0, 7 * SR)), 5 * SR, SR, snr_db=20.0, salt=40 + i)
          for i in range(0, 20, 2)]
    out = {}
    for mode in ("atomic", "sort", "ballot"):
        eng = Engine(SR)
        try:
            eng.force("k4_build", {"atomic": 2, "sort": 1, "ballot": 4}[mode])
            pcm = torch.empty(len(tracks) * n, dtype=torch.float32, device="cuda")
            eng.synth(pcm.data_ptr(), tracks, np.zeros(len(tracks), np.int64), n)
            eng.extract_device(pcm.data_ptr(), np.arange(len(tracks) + 1, dtype=np.int64) * n)
            eng.index_add_extracted(tracks)
            eng.index_remove(int(tracks[4]))
            eng.index_remove(int(tracks[10]))
            eng.index_finalize()
            recs = [O.fingerprint(q, HOP) for q in qs]
            out[mode] = (eng.index_stats(), eng.query(recs))
        finally:
            eng.close()
    (sa, ra), (ss, rs), (sr, rr) = out["atomic"], out["sort"], out["ballot"]
    assert sr == ss and all(np.array_equal(a, b) for a, b in zip(rr, rs))  # one-atomic rank == ballot rank
    assert sa["live"] == ss["live"] > 0 and sa["postings"] == ss["postings"]
    assert any(len(r) for r in rs)
    for q, (a, b) in enumerate(zip(ra, rs)):
        assert np.array_equal(a, b), f"query {q}: rows differ between the builds"
        assert not np.isin(b[:, 1] if len(b) else [], [tracks[4], tracks[10]]).any()



@pytest.mark.parametrize("removed", [False, True])
def test_sort_build_many_column_groups(removed):
    """The radix build over more than one column-scan group (> 256 tiles of 4096 postings, ~1.4 M postings here), with
    and without tombstones (the templated first pass): rows equal the atomic counting build's for 48 queries."""
    import torch

    n = SR * 12
    tracks = np.arange(600, dtype=np.uint32) * 3 + 1
    rng = np.random.default_rng(11)
    pick = rng.choice(len(tracks), 48, replace=False)
    qs = [synth.synth(int(tracks[i]), int(rng.integers(0, 7 * SR)), 5 * SR, SR, snr_db=20.0, salt=60 + int(i))
          for i in pick]
    recs = [O.fingerprint(q, HOP) for q in qs]
    out = {}
    for mode in ("sort", "atomic"):
        eng = Engine(SR)
        try:
            eng.force("k4_build", {"sort": 1, "atomic": 2}[mode])
            pcm = torch.empty(200 * n, dtype=torch.float32, device="cuda")
            for b0 in range(0, len(tracks), 200):
                tr = tracks[b0:b0 + 200]
                eng.synth(pcm.data_ptr(), tr, np.zeros(len(tr), np.int64), n)
                eng.extract_device(pcm.data_ptr(), np.arange(len(tr) + 1, dtype=np.int64) * n)
                eng.index_add_extracted(tr)
            if removed:
                for i in pick[:5]:
                    eng.index_remove(int(tracks[i]))
            eng.index_finalize()
            st = eng.index_stats()
            assert st["postings"] > 256 * 4096
            out[mode] = (st, eng.query(recs))
        finally:
            eng.close()
    (ss, rs), (sr, rr) = out["sort"], out["atomic"]
    assert ss["live"] == sr["live"] and ss["postings"] == sr["postings"]
    assert all(np.array_equal(a, b) for a, b in zip(rs, rr))
    hits = [int(r[0, 1]) if len(r) else None for r in rs]
    gone = {int(tracks[i]) for i in pick[:5]} if removed else set()
    assert sum(h == int(tracks[i]) for h, i in zip(hits, pick) if int(tracks[i]) not in gone) >= 40
    assert not any(h in gone for h in hits if h is not None)


def _bucket_key_np(h):
    """Host mirror of aidfp_layout.h bucket_key (the CSR's key permutation of the 26 hash bits)."""
    h = h.astype(np.uint32)
    return ((((h >> 22) & 0xFF) << 18) | ((h >> 30) << 16) | (((h >> 12) & 0x7F) << 9) | (((h >> 19) & 0x7) << 6) |
            (h & 0x3F)).astype(np.uint32)


def _csr_mirror(post, removed):
    """The CSR K4 must build from stored postings [n, 3] (hash, track, t): live postings stably sorted by bucket key
    (a bucket keeps arrival order), values track | t << 32, offsets[k] = live postings with key < k."""
    live = ~np.isin(post[:, 1], np.asarray(list(removed), dtype=np.uint32))
    p = post[live]
    keys = _bucket_key_np(p[:, 0])
    order = np.argsort(keys, kind="stable")
    posts = p[order, 1].astype(np.uint64) | (p[order, 2].astype(np.uint64) << np.uint64(32))
    counts = np.bincount(keys, minlength=1 << 26)
    offs = np.zeros((1 << 26) + 1, np.uint32)
    offs[1:] = np.cumsum(counts).astype(np.uint32)
    return offs, posts


@pytest.mark.parametrize("mode", ["sort", "ballot"])
def test_csr_layout_equals_stable_mirror(mode):
    """The built CSR itself, not only the rows queries read from it: the hand-written radix build (its default rank,
    one LDS atomic per posting; and the ballot-matched rank, force 4) lays out
    exactly the stable key sort of the stored postings (arrival order inside a bucket), with
    removed tracks' postings dropped and offsets equal to the key histogram's prefix sums; over more than one K4
    tile and column group (~1.4 M postings)."""
    import torch

    n = SR * 12
    tracks = np.arange(600, dtype=np.uint32) * 5 + 2
    removed = {int(tracks[3]), int(tracks[300]), int(tracks[599])}
    eng = Engine(SR)
    try:
        eng.force("k4_build", {"sort": 1, "ballot": 4}[mode])
        pcm = torch.empty(200 * n, dtype=torch.float32, device="cuda")
        for b0 in range(0, len(tracks), 200):
            tr = tracks[b0:b0 + 200]
            eng.synth(pcm.data_ptr(), tr, np.zeros(len(tr), np.int64), n)
            eng.extract_device(pcm.data_ptr(), np.arange(len(tr) + 1, dtype=np.int64) * n)
            eng.index_add_extracted(tr)
        for t in sorted(removed):
            eng.index_remove(t)
        eng.index_finalize()
        post = eng.index_export()
        offs, posts = eng.index_csr()
    finally:
        eng.close()
    assert len(post) > 256 * 4096
    ref_offs, ref_posts = _csr_mirror(post, removed)
    assert len(posts) == len(ref_posts)
    bad = np.flatnonzero(posts != ref_posts)
    assert len(bad) == 0, f"{len(bad)} CSR postings out of place, first at {bad[:5]}"
    assert np.array_equal(offs, ref_offs)


def test_rocprim_ab_not_in_product_library():
    """The rocPRIM sort is an A/B reference of the diagnostic variant build only: the product
    library refuses k4_build 3 and links no rocPRIM code."""
    from aidfp._lib import EngineError

    eng = Engine(SR)
    try:
        with pytest.raises(EngineError):
            eng.force("k4_build", 3)
    finally:
        eng.close()


def test_csr_export_needs_a_finalized_index():
    """aid_index_csr_export refuses a stale index (AID_ERR_STATE) and returns an empty CSR for an empty one."""
    from aidfp._lib import AID_ERR_STATE, EngineError

    eng = Engine(SR)
    try:
        eng.index_finalize()
        offs, posts = eng.index_csr()
        assert len(posts) == 0 and offs[0] == 0 and offs[-1] == 0
        rec = O.fingerprint(synth.synth(3, 0, 5 * SR, SR), HOP)
        eng.index_add_records(3, rec)
        with pytest.raises(EngineError) as e:
            eng.index_csr(offsets=False)
        assert e.value.code == AID_ERR_STATE
        eng.index_finalize()
        _, posts = eng.index_csr(offsets=False)
        assert len(posts) == len(rec)
    finally:
        eng.close()


@pytest.mark.parametrize("mode", ["sort", "ballot"])
@pytest.mark.parametrize("n", [1, 100, 4096, 4097, 3 * 4096 + 5])
def test_csr_layout_small_and_tile_edges(mode, n):
    """K4 at the tile edges (a single posting, a partial tile, exactly one tile, one posting past it, several tiles
    and a remainder), random hashes with many collisions and one removed track: the CSR equals the stable mirror."""
    rng = np.random.default_rng(n)
    h = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    h[rng.random(n) < 0.5] = np.uint32(0x12345678)  # half the postings in one bucket: long runs across tiles
    tr = rng.integers(0, 7, n).astype(np.uint32)
    t = rng.integers(0, 5000, n).astype(np.uint32)
    eng = Engine(SR)
    try:
        eng.force("k4_build", {"sort": 1, "ballot": 4}[mode])
        eng.index_add_postings(h.ctypes.data, tr.ctypes.data, t.ctypes.data, n, device=False)
        removed = {3} if n > 1 else set()
        for r in removed:
            if (tr == r).any():
                eng.index_remove(r)
            else:
                removed = set()
        eng.index_finalize()
        offs, posts = eng.index_csr()
        post = eng.index_export()
    finally:
        eng.close()
    ref_offs, ref_posts = _csr_mirror(post, removed)
    assert np.array_equal(posts, ref_posts)
    assert np.array_equal(offs, ref_offs)


def test_async_append_equals_per_clip_records(tmp_path):
    """aid_index_add_extracted appends without waiting for its batch's counts (offsets scanned on the device, the
    new total read back by the next reader; engine.cpp settle_postings): batches of every size, a silent clip and
    one shorter than a frame, readers and a host append between them, and batches beyond the planes' headroom
    (the growth path, counts read back first) store exactly each clip's records under its track, in call order."""
    sr = 16000
    rng = np.random.default_rng(3)
    with Engine(sr) as eng:
        want, tid = [], 100

        def rows(t, r):
            return np.stack([(r & np.uint64(0xFFFFFFFF)).astype(np.uint32), np.full(len(r), t, np.uint32),
                             (r >> np.uint64(32)).astype(np.uint32)], axis=1)

        for b, k in enumerate([1, 4, 2, 7, 1, 3, 24, 2, 1]):
            clips = [synth.synth(tid + j, int(rng.integers(0, 5 * sr)), int(rng.integers(2 * sr, 9 * sr)), sr,
                                 snr_db=30.0, salt=b) for j in range(k)]
            if b == 2:
                clips += [np.zeros(3 * sr, np.float32), np.zeros(100, np.float32)]
            recs = eng.extract_host(clips)
            tracks = np.arange(tid, tid + len(clips), dtype=np.uint32)
            eng.index_add_extracted(tracks)
            want += [rows(t, r) for t, r in zip(tracks, recs)]
            tid += len(clips)
            if b == 3:
                assert eng.index_stats()["postings"] == sum(map(len, want))
            if b == 4:
                eng.index_add_records(tid, recs[0])
                want.append(rows(tid, recs[0]))
                tid += 1
            if b == 5:
                assert np.array_equal(eng.index_export(), np.concatenate(want))
            if b == 7:
                path = tmp_path / "mid.aidfp"
                eng.index_save(str(path))
                with Engine(sr) as e2:
                    e2.index_load(str(path))
                    assert np.array_equal(e2.index_export(), np.concatenate(want))
        post = eng.index_export()
        assert np.array_equal(post, np.concatenate(want))
        eng.index_finalize()
        assert eng.index_stats()["live"] == len(post)
        eng.index_reset()
        assert eng.index_stats()["postings"] == 0
        recs = eng.extract_host([synth.synth(7, 0, 4 * sr, sr), synth.synth(8, 0, 5 * sr, sr)])
        eng.index_add_extracted(np.array([7, 8], np.uint32))
        assert np.array_equal(eng.index_export(), np.concatenate([rows(7, recs[0]), rows(8, recs[1])]))


@pytest.mark.parametrize("path", [0, 1, 2])
def test_match_v1_golden_fixture_on_gpu(path):
    """The committed FPSPEC v1 match vectors (tests/golden/oracle_match_v1.*) through the engine: the fixture's postings
    added as raw postings, its query records matched on the automatic, LDS and global paths -- rows equal the
    fixture's (distinct anchor frames, min_match 10)."""
    import json
    from pathlib import Path

    gdir = Path(__file__).resolve().parent / "golden"
    g = np.load(gdir / "oracle_match_v1.npz")
    meta = json.loads((gdir / "oracle_match_v1.json").read_text())
    post = np.ascontiguousarray(g["postings"])
    eng = Engine(meta["sr"])
    try:
        h, t, tm = (np.ascontiguousarray(post[:, k]) for k in range(3))
        eng.index_add_postings(h.ctypes.data, t.ctypes.data, tm.ctypes.data, len(post), device=False)
        eng.index_finalize()
        if path:
            eng.force("k5_path", path)
        recs = [g[f"rec_{i}"] for i in range(len(meta["queries"]))]
        got = eng.query(recs)
        for i, r in enumerate(got):
            assert np.array_equal(r, g[f"rows_mm10_{i}"]), (i, r, g[f"rows_mm10_{i}"])
    finally:
        eng.close()
