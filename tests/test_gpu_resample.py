"""GPU PCM front-end (K6 `resample`, FPSPEC 8) through the C ABI: bit-exact vs the CPU oracle
(oracle/fp_resample.c, itself pinned to scipy.signal.resample_poly by test_resample_oracle.py),
the streaming range form, and a 48 kHz stereo stream identified against a 16 kHz index -- the
reference's own configuration (UI records 48 kHz, the Olaf index is 16 kHz: decode.py:41-60,
fingerprint.py:10)."""

import numpy as np
import pytest
import torch

import oracle as O
from aidfp import synth
from aidfp.engine import Engine
from aidfp.stream import StreamIdentifier

pytestmark = pytest.mark.gpu
RATES = [(48000, 16000), (48000, 44100), (44100, 16000), (16000, 48000), (44100, 48000), (22050, 16000),
         (96000, 44100), (8000, 44100), (16000, 16000), (44101, 48000)]


def _gpu_resample(eng, x, sr_in, sr_out):
    ch = 1 if x.ndim == 1 else 2
    src = torch.from_numpy(np.ascontiguousarray(x, np.float32).reshape(-1)).cuda()
    m = eng.resample_len(len(x), sr_in, sr_out)
    dst = torch.full((max(m, 1),), float("nan"), dtype=torch.float32, device="cuda")
    got = eng.resample(src.data_ptr(), len(x), ch, sr_in, sr_out, dst.data_ptr(), m)
    torch.cuda.synchronize()
    assert got == m
    return dst[:m].cpu().numpy()


@pytest.mark.parametrize("sr_in,sr_out", RATES)
def test_resample_bit_exact(gpu_engine, sr_in, sr_out):
    rng = np.random.default_rng(sr_in * 7 + sr_out)
    for n in (1, 5, 999, 2 * sr_in + 17):
        for stereo in (False, True):
            x = (rng.standard_normal((n, 2) if stereo else n) * 0.4).astype(np.float32)
            if sr_in == sr_out and stereo:
                ref = O.resample(x, sr_in, sr_out)
            else:
                ref = O.resample(x, sr_in, sr_out)
            got = _gpu_resample(gpu_engine, x, sr_in, sr_out)
            assert got.shape == ref.shape
            assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (sr_in, sr_out, n, stereo)


def test_resample_range_chunks_equal_whole(gpu_engine):
    sr_in, sr_out = 48000, 44100
    up, down, hl, J = gpu_engine.resample_plan(sr_in, sr_out)
    rng = np.random.default_rng(5)
    x = (rng.standard_normal((sr_in * 3, 2)) * 0.3).astype(np.float32)
    ref = O.resample(x, sr_in, sr_out)
    out = torch.empty(len(ref), dtype=torch.float32, device="cuda")
    m = 0
    cuts = sorted(rng.integers(1, len(ref), size=11).tolist()) + [len(ref)]
    for end in cuts:
        if end <= m:
            continue
        lo = max(0, (m * down + hl) // up - (J - 1))          # first input the chunk reads
        hi = min(len(x), ((end - 1) * down + hl) // up + 1)   # one past the last
        src = torch.from_numpy(np.ascontiguousarray(x[lo:hi]).reshape(-1)).cuda()
        gpu_engine.resample_range(src.data_ptr(), lo, hi - lo, 2, sr_in, sr_out, m, end - m,
                                  out.data_ptr() + 4 * m)
        torch.cuda.synchronize()
        m = end
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_resample_errors(gpu_engine):
    from aidfp._lib import EngineError

    src = torch.zeros(2001, dtype=torch.float32, device="cuda")
    dst = torch.zeros(1000, dtype=torch.float32, device="cuda")
    with pytest.raises(EngineError):  # capacity
        gpu_engine.resample(src.data_ptr(), 2000, 1, 16000, 48000, dst.data_ptr(), 1000)
    with pytest.raises(EngineError):  # stereo source must be 8-byte aligned
        gpu_engine.resample(src.data_ptr() + 4, 1000, 2, 48000, 16000, dst.data_ptr(), 1000)
    with pytest.raises(EngineError):  # bad rate
        gpu_engine.resample(src.data_ptr(), 10, 1, 0, 16000, dst.data_ptr(), 1000)


def test_stream_resampled_buffer_equals_whole_stream():
    """Chunked stream resampling (with compactions) == resampling the whole stream at once."""
    with Engine(16000) as eng:
        rng = np.random.default_rng(9)
        st = (rng.standard_normal((48000 * 40, 2)) * 0.3).astype(np.float32)
        ref = O.resample(st, 48000, 16000)
        sid = StreamIdentifier(eng, window_s=5.0, hop_s=2.5, capacity_s=12.0, stream_sr=48000)
        a = 0
        held = []
        while a < len(st):
            b = min(len(st), a + int(rng.integers(1, 30000)))
            sid.push(st[a:b])
            a = b
            held.append((sid.base, sid.mono_history()))
        for base, h in held[-3:]:
            assert len(h) > 0
            assert np.array_equal(h.view(np.uint32), ref[base:base + len(h)].view(np.uint32))
        # everything whose filter window is complete was produced
        up, down, hl, _ = eng.resample_plan(48000, 16000)
        assert sid.m_next == (len(st) * up - 1 - hl) // down + 1


def test_48k_stereo_stream_against_16k_index():
    """The reference's deployment shape: the catalog ingested from 44.1 kHz files decoded to 16 kHz
    (ffmpeg -ar 16000, decode.py:41-60; here K6 per track), queried by 48 kHz stereo capture
    (AudioRecorder.svelte:86-106) downmixed and resampled to 16 kHz (fingerprint.py:10).

    Parity: every window's rows equal those of the CPU route (oracle resampling of the whole
    stream -> window slice -> oracle fingerprint -> query). Identification: top-1 >= 0.98 on windows
    inside a segment (scripts/eval_exact.py:46-54's clean target). The capture shares nothing
    sample-exact with the index (other rate, other noise), so this needs the v2 generator's note
    envelopes: with stationary v0 notes the peak frame on a note's plateau is decided by noise and
    top-1 was 0.66-0.74."""
    with Engine(16000) as eng:
        from aidfp.catalog import ingest_synthetic

        ingest_synthetic(eng, np.arange(30, dtype=np.uint32), 30.0, source_sr=44100)
        order = [4, 21, 11]
        seg = 30 * 48000
        L = np.concatenate([synth.synth(t, 0, seg, 48000, snr_db=30.0, salt=1) for t in order])
        R = np.concatenate([synth.synth(t, 0, seg, 48000, snr_db=30.0, salt=2) for t in order])
        st = np.stack([L, R], axis=1)
        sid = StreamIdentifier(eng, capacity_s=20.0, stream_sr=48000)
        res = []
        for a in range(0, len(st), 24000):
            res += sid.push(st[a:a + 24000])
        mono = O.resample(st, 48000, 16000)
        recs = [O.fingerprint(mono[int(round(r.start_s * 16000)):int(round(r.start_s * 16000)) + sid.win], eng.hop)
                for r in res]
        ref_rows = eng.query(recs)
        for r, ref in zip(res, ref_rows):
            assert np.array_equal(r.rows, ref), r.start_s
        inside = [r for r in res if int(r.start_s // 30) == int((r.start_s + 5.0 - 1e-9) // 30)]
        assert len(inside) >= 25
        hits = [r.best_track == order[int(r.start_s // 30)] for r in inside]
        wrong = [(r.start_s, r.best_track, int(r.rows[0, 0]) if len(r.rows) else 0) for r, h in zip(inside, hits) if not h]
        assert np.mean(hits) >= 0.98, (np.mean(hits), wrong)
