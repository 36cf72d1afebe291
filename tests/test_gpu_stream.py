"""Streaming front end on the GPU: downmix bit-exact vs numpy binary32, and the
window scheduler identifying tracks of a stereo stream (config 5 shape)."""

import numpy as np
import pytest
import torch

from aidfp import synth
from aidfp.engine import Engine
from aidfp.stream import StreamIdentifier

pytestmark = pytest.mark.gpu
SR = 48000


def test_downmix_bit_exact(gpu_engine):
    rng = np.random.default_rng(0)
    for n in (1, 2, 7, 1000, 48001):
        x = rng.standard_normal((n, 2)).astype(np.float32)
        src = torch.from_numpy(x.reshape(-1)).cuda()
        dst = torch.empty(n, dtype=torch.float32, device="cuda")
        gpu_engine.downmix(src.data_ptr(), n, dst.data_ptr())
        torch.cuda.synchronize()
        ref = (x[:, 0] + x[:, 1]) * np.float32(0.5)
        assert np.array_equal(dst.cpu().numpy(), ref)


def test_stream_windows_identify_segments():
    with Engine(SR) as eng:
        from aidfp.catalog import ingest_synthetic

        ingest_synthetic(eng, np.arange(40, dtype=np.uint32), 30.0)
        seg = 30 * SR
        order = [3, 17, 29]
        L = np.concatenate([synth.synth(t, 0, seg, SR, snr_db=30.0, salt=1) for t in order])
        R = np.concatenate([synth.synth(t, 0, seg, SR, snr_db=30.0, salt=2) for t in order])
        st = np.stack([L, R], axis=1)
        sid = StreamIdentifier(eng, capacity_s=20.0)  # forces buffer compaction
        res = []
        for a in range(0, len(st), 12345):  # odd chunk sizes exercise the carry
            res += sid.push(st[a:a + 12345])
        assert len(res) == int((len(st) / SR - 5.0) // 2.5) + 1
        for r in res:
            s0 = int(round(r.start_s * SR))
            if s0 // seg == (s0 + sid.win - 1) // seg:
                assert r.best_track == order[s0 // seg]


def _stereo_streams(tracks_per_stream, seg_s, sr, salt0=0):
    seg = int(seg_s * sr)
    out = []
    for i, order in enumerate(tracks_per_stream):
        L = np.concatenate([synth.synth(int(t), 0, seg, sr, snr_db=30.0, salt=salt0 + 2 * i + 1) for t in order])
        R = np.concatenate([synth.synth(int(t), 0, seg, sr, snr_db=30.0, salt=salt0 + 2 * i + 2) for t in order])
        out.append(np.stack([L, R], axis=1))
    return np.stack(out)  # [S, n, 2]


@pytest.mark.parametrize("device_chunks", [True, False])
def test_stream_bank_equals_single_streams(device_chunks):
    """StreamBank (one K6 launch + one aid_query_windows call per push for all streams) gives every stream exactly
    the windows and rows of its own StreamIdentifier (per-stream K6 + per-stream queries), with buffer compaction
    and chunks that are not a multiple of the hop."""
    from aidfp.catalog import ingest_synthetic
    from aidfp.stream import StreamBank

    with Engine(16000) as eng:
        ingest_synthetic(eng, np.arange(30, dtype=np.uint32), 30.0, source_sr=44100)
        orders = [[3, 17], [29, 4], [11, 11], [0, 25], [7, 8]]
        st = _stereo_streams(orders, 12.0, SR)  # 24 s per stream
        bank = StreamBank(eng, len(orders), stream_sr=SR, capacity_s=12.0)  # forces compaction of both buffers
        singles = [StreamIdentifier(eng, capacity_s=12.0, stream_sr=SR) for _ in orders]
        step = 50000
        got = [[] for _ in orders]
        want = [[] for _ in orders]
        for a in range(0, st.shape[1], step):
            chunk = st[:, a:a + step]
            res = bank.push(torch.from_numpy(np.ascontiguousarray(chunk)).cuda() if device_chunks else chunk)
            for i in range(len(orders)):
                got[i] += res[i]
                want[i] += singles[i].push(chunk[i])
        for i in range(len(orders)):
            assert len(got[i]) == len(want[i]) == int((st.shape[1] / SR - 5.0) // 2.5) + 1
            for g, w in zip(got[i], want[i]):
                assert g.start_s == w.start_s and np.array_equal(g.rows, w.rows), (i, g.start_s)
        # and the windows inside a 12 s segment name its track
        hits = total = 0
        for i, order in enumerate(orders):
            for r in got[i]:
                a, b = r.start_s, r.start_s + 5.0
                if int(a // 12.0) == int((b - 1e-9) // 12.0):
                    total += 1
                    hits += r.best_track == order[int(a // 12.0)]
        assert total >= 10 and hits == total


def test_resample_batch_equals_single_streams(gpu_engine):
    """aid_resample_batch: n streams in one launch = n aid_resample_range calls, bit for bit (48k -> 16k and
    48k -> 44.1k stereo, 44.1k -> 16k mono)."""
    rng = np.random.default_rng(4)
    for sr_in, sr_out, ch in ((48000, 16000, 2), (48000, 44100, 2), (44100, 16000, 1)):
        S, n, m0, cnt = 3, 30011, 101, 7000
        x = rng.standard_normal((S, n * ch + 6)).astype(np.float32)  # stride > one stream's samples
        src = torch.from_numpy(x).cuda()
        out_b = torch.zeros(S, cnt + 5, dtype=torch.float32, device="cuda")
        gpu_engine.resample_batch(src.data_ptr(), x.shape[1], S, 17, n, ch, sr_in, sr_out, m0, cnt, out_b.data_ptr(),
                                  cnt + 5)
        for i in range(S):
            one = torch.zeros(cnt, dtype=torch.float32, device="cuda")
            gpu_engine.resample_range(src[i].data_ptr(), 17, n, ch, sr_in, sr_out, m0, cnt, one.data_ptr())
            torch.cuda.synchronize()
            assert torch.equal(out_b[i, :cnt], one), (sr_in, sr_out, ch, i)
            assert not out_b[i, cnt:].any()


def test_resample_batch_split_equals_whole(gpu_engine):
    """aid_resample_batch_split: a two-part input (the last h frames before stream frame k from a history buffer,
    frames k.. from the chunk where it lies) gives aid_resample_batch's outputs over the whole input, bit for bit."""
    rng = np.random.default_rng(9)
    for sr_in, sr_out, ch in ((48000, 16000, 2), (48000, 44100, 2), (44100, 16000, 1)):
        up, down, hl, J = gpu_engine.resample_plan(sr_in, sr_out)
        S, N, k, h = 3, 40000, 20001, J + 3
        x = rng.standard_normal((S, N * ch + 4)).astype(np.float32)
        whole = torch.from_numpy(x).cuda()
        hist = torch.from_numpy(np.ascontiguousarray(x[:, (k - h) * ch: k * ch])).cuda()
        cur = whole[:, k * ch:]  # in place: a strided view of the whole input
        m0 = -(-((k - h + J - 1) * up - hl) // down)  # first output whose window starts at or after frame k - h
        cnt = (N * up - 1 - hl) // down + 1 - m0       # through the last output with its inputs in range
        a = torch.zeros(S, cnt, dtype=torch.float32, device="cuda")
        b = torch.zeros(S, cnt, dtype=torch.float32, device="cuda")
        gpu_engine.resample_batch(whole.data_ptr(), x.shape[1], S, 0, N, ch, sr_in, sr_out, m0, cnt, a.data_ptr(), cnt)
        gpu_engine.resample_batch_split(hist.data_ptr(), h * ch, h, cur.data_ptr(), x.shape[1], S, k, N - k, ch, sr_in,
                                        sr_out, m0, cnt, b.data_ptr(), cnt)
        torch.cuda.synchronize()
        assert torch.equal(a, b), (sr_in, sr_out, ch)


@pytest.mark.parametrize("steps", [(37, 1, 5000, 48000), (120000,)])
def test_stream_bank_chunk_sizes(steps):
    """StreamBank keeps only the last J - 1 input frames between pushes (the chunk is read in place): pushes of 1,
    37 and 5000 frames (shorter than the filter: the history comes partly from earlier chunks) and whole 2.5 s
    pushes give exactly the windows of a per-stream StreamIdentifier."""
    from aidfp.catalog import ingest_synthetic
    from aidfp.stream import StreamBank

    with Engine(16000) as eng:
        ingest_synthetic(eng, np.arange(12, dtype=np.uint32), 30.0, source_sr=44100)
        orders = [[3, 7], [11, 2]]
        st = _stereo_streams(orders, 6.0, SR, salt0=40)  # 12 s per stream
        dev = torch.from_numpy(st).cuda()
        bank = StreamBank(eng, len(orders), stream_sr=SR)
        singles = [StreamIdentifier(eng, stream_sr=SR) for _ in orders]
        got = [[] for _ in orders]
        want = [[] for _ in orders]
        a = i = 0
        while a < st.shape[1]:
            step = steps[i % len(steps)]
            i += 1
            res = bank.push(dev[:, a:a + step])
            for j in range(len(orders)):
                got[j] += res[j]
                want[j] += singles[j].push(st[j, a:a + step])
            a += step
        assert bank.hist_n <= bank.J - 1
        for j in range(len(orders)):
            assert len(got[j]) == len(want[j]) == int((st.shape[1] / SR - 5.0) // 2.5) + 1
            for g, w in zip(got[j], want[j]):
                assert g.start_s == w.start_s and np.array_equal(g.rows, w.rows), (j, g.start_s)


def test_stream_bank_equals_oracle_route():
    """The production streaming path: StreamBank with 6 live 48 kHz stereo streams in lockstep
    against a 16 kHz index ingested from 44.1 kHz sources (the reference's deployment shape), pushed in 1.37 s
    chunks so windows straddle chunk boundaries; the first 4 streams' windows equal the oracle route -- host
    downmix, oracle/fp_resample.c 48k -> 16k, oracle/fp_oracle.c per window, oracle/fp_match.c over this index's
    postings (bench.stream_parity, the check the bench's stream key runs)."""
    import bench
    from aidfp.catalog import ingest_synthetic
    from aidfp.stream import StreamBank

    SSR, QSR = 16000, 48000
    with Engine(SSR) as eng:
        ingest_synthetic(eng, np.arange(60, dtype=np.uint32), 30.0, batch=64, source_sr=44100, local=True)
        eng.index_finalize()
        S, n_seg, seg = 6, 2, 12 * QSR
        seg_tracks = np.random.default_rng(3).integers(0, 60, (S, n_seg)).astype(np.uint32)
        stereo = torch.empty(S, n_seg * seg, 2, dtype=torch.float32, device="cuda")
        tmp = torch.empty(S * n_seg * seg, dtype=torch.float32, device="cuda")
        for ch in range(2):
            eng.synth(tmp.data_ptr(), seg_tracks.ravel(), np.zeros(S * n_seg, np.int64), seg,
                      noise_a=synth.noise_halfwidth(30.0), salt=11 + ch, sample_rate=QSR)
            stereo[:, :, ch] = tmp.view(S, n_seg * seg)
        torch.cuda.synchronize()
        bank = StreamBank(eng, S, stream_sr=QSR)
        res = [[] for _ in range(S)]
        chunk = int(1.37 * QSR)
        for a in range(0, stereo.shape[1], chunk):
            r = bank.push(stereo[:, a:a + chunk])
            for i in range(S):
                res[i] += r[i]
        assert all(len(res[i]) == int((n_seg * 12.0 - 5.0) // 2.5) + 1 for i in range(S))
        assert sum(len(w.rows) > 0 for i in range(S) for w in res[i]) > 0
        par = bench.stream_parity(eng, stereo, seg_tracks, res, 4, torch, max_windows=8)
    assert par["windows"] == 4 * 8
    assert par["bit_exact"], par


def test_stream_bank_pipelined_equals_sync():
    """StreamBank.push_submit (aid_query_windows_submit / _collect): submitting push N + 1 before
    collecting push N gives every push exactly the rows of the synchronous push()."""
    from aidfp.catalog import ingest_synthetic
    from aidfp.stream import StreamBank

    SSR, QSR = 16000, 48000
    with Engine(SSR) as eng:
        ingest_synthetic(eng, np.arange(40, dtype=np.uint32), 30.0, batch=64, source_sr=44100, local=True)
        eng.index_finalize()
        S, seg = 5, 14 * QSR
        tr = np.random.default_rng(9).integers(0, 40, S).astype(np.uint32)
        stereo = torch.empty(S, seg, 2, dtype=torch.float32, device="cuda")
        tmp = torch.empty(S * seg, dtype=torch.float32, device="cuda")
        for ch in range(2):
            eng.synth(tmp.data_ptr(), tr, np.zeros(S, np.int64), seg, noise_a=synth.noise_halfwidth(30.0),
                      salt=21 + ch, sample_rate=QSR)
            stereo[:, :, ch] = tmp.view(S, seg)
        chunk = int(1.7 * QSR)
        sync_bank, pipe_bank = StreamBank(eng, S, stream_sr=QSR), StreamBank(eng, S, stream_sr=QSR)
        want, got, pending = [], [], None
        for a in range(0, seg, chunk):
            want.append(sync_bank.push(stereo[:, a:a + chunk]))
            p = pipe_bank.push_submit(stereo[:, a:a + chunk])
            if pending is not None:
                got.append(pending.collect())
            pending = p
        got.append(pending.collect())
        assert sum(len(w) for push in want for w in push) > 0
        for w, g in zip(want, got):
            for ws, gs in zip(w, g):
                assert [x.start_s for x in ws] == [x.start_s for x in gs]
                for x, y in zip(ws, gs):
                    assert np.array_equal(x.rows, y.rows)


def test_query_windows_submit_collect_with_fallbacks():
    """Two tickets in flight, collected out of order, and queries the fast match path hands back (min_match 1: more
    candidate tracks than its row staging holds): rows equal aid_query_windows' (which takes the global path for them
    too) and the oracle's."""
    import oracle as O
    from aidfp.catalog import ingest_synthetic

    SSR = 16000
    with Engine(SSR, min_match=1) as eng:
        ingest_synthetic(eng, np.arange(1200, dtype=np.uint32), 30.0, batch=256, source_sr=44100, local=True)
        eng.index_finalize()
        n = 20 * SSR
        pcm = torch.empty(4 * n, dtype=torch.float32, device="cuda")
        eng.synth(pcm.data_ptr(), np.array([3, 77, 150, 299], np.uint32), np.zeros(4, np.int64), n,
                  noise_a=synth.noise_halfwidth(20.0), salt=5, sample_rate=SSR)
        st = np.array([0, 7 * SSR, n + 3 * SSR, 2 * n + 11, 3 * n + 5 * SSR], np.int64)
        en = st + np.array([5, 5, 5, 9, 5], np.int64) * SSR
        eng.match_stats(reset=True)
        want = eng.query_windows(pcm.data_ptr(), st, en)
        a = eng.query_windows_submit(pcm.data_ptr(), st[:3], en[:3])
        b = eng.query_windows_submit(pcm.data_ptr(), st[3:], en[3:])
        gb, ga = b.collect(), a.collect()
        ms = eng.match_stats()
        # the case under test: the LDS path handed some queries back (every bucket is hot at min_match 1, so its
        # tables fill) and collect answered them on the global path
        assert sum(ms[k] for k in ("fallback_table", "fallback_distinct", "fallback_tracks", "fallback_rows")) > 0, ms
        for w, g in zip(want, ga + gb):
            assert np.array_equal(w, g)
        post = eng.index_export()
        host = pcm.cpu().numpy()
        for k in range(len(st)):
            rec = O.fingerprint(host[st[k]:en[k]], 256)
            assert np.array_equal(want[k], O.query(post, rec, min_match=1, max_rows=eng.max_results))
