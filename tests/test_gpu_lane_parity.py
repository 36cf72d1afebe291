"""bench.py's config-4 parity check (catalog.exact_lane.parity) on a small catalog: the sampled clips' window
records, K5 rows on every path and the batched lane's rows against the all-oracle lane (oracle/fp_oracle.c +
oracle/fp_match.c + aidfp.exact's per-window path; reference app/search/exact.py:132-293). The bench runs the
same function at the configured scale (100k tracks); here the catalog is small enough for a test."""

import types

import numpy as np
import pytest

import bench
from bench_match import CATEGORIES, run_batches

pytestmark = pytest.mark.gpu
SR = 44100
N_TRACKS = 200


@pytest.fixture(scope="module")
def catalog():
    from aidfp.catalog import ingest_synthetic
    from aidfp.engine import Engine

    eng = Engine(SR)
    ingest_synthetic(eng, np.arange(N_TRACKS, dtype=np.uint32), 30.0, batch=128)
    eng.index_finalize()
    yield eng
    eng.close()


@pytest.mark.parametrize("category", ["noise20", "clean"])
def test_lane_parity_small_catalog(catalog, category):
    import torch

    eng = catalog
    rng = np.random.default_rng(3)
    n_pos, n_neg = 90, 10
    truth = np.concatenate([rng.integers(0, N_TRACKS, n_pos), np.arange(n_neg) + N_TRACKS + 10**6]).astype(np.uint32)
    starts = np.concatenate([rng.integers(0, 25 * SR, n_pos), np.zeros(n_neg, np.int64)]).astype(np.int64)
    clip_n = 5 * SR
    a = types.SimpleNamespace(batch=64, sr=SR)  # two lane calls: the kept rows come from both
    pcm = torch.empty(64 * clip_n, dtype=torch.float32, device="cuda")
    sel = np.array([0, 5, 63, 64, 70, 89, 90, 95, 99], dtype=np.int64)
    res, _ = run_batches(a, eng, truth, starts, n_pos, CATEGORIES[category], pcm, clip_n, False, keep=sel)
    del pcm
    kept = res.pop("kept")
    assert sorted(kept) == sel.tolist()
    par = bench.lane_parity(eng, truth, starts, n_pos, sel, kept, CATEGORIES[category], torch)
    assert par["records_bit_exact"], par
    assert par["rows_bit_exact"], par["k5_paths"]
    assert par["lane_equal"], par
    assert par["negatives"] == 3 and par["windows"] == 3 * len(sel)
    assert par["k5_paths"]["global"]["queries_global"] == par["windows"]
    assert par["k5_paths"]["lds"]["queries_lds"] == par["windows"]
    # the positives were found (the check is not vacuous)
    assert sum(len(kept[int(q)]) > 0 for q in sel if q < n_pos) >= 5


def test_index_checksum_equals_host_mirror(catalog):
    """aid_index_checksum (device) equals its host mirror over the exported postings, whole and by range."""
    from aidfp.catalog import checksum_np

    eng = catalog
    post = eng.index_export()
    assert eng.index_checksum() == checksum_np(post)
    n = len(post)
    assert eng.index_checksum(n // 3, n // 2) == checksum_np(post[n // 3: n // 3 + n // 2])
    assert eng.index_checksum(n, 0) == 0


def test_shard_parity_small_catalog(catalog):
    """bench.shard_parity: the oracle's fingerprints of sampled tracks of every (pretend) rank's shard equal this
    index's postings of those tracks."""
    import torch

    par = bench.shard_parity(catalog, np.arange(N_TRACKS, dtype=np.uint32), 30.0, 3, torch, per_rank=4)
    assert par["bit_exact"], par
    assert par["tracks_checked"] == 12 and par["postings_checked"] > 1000
