"""GPU parity: K1-K3 through the C ABI vs the CPU oracle (bit-exact), and the
GPU log-magnitude vs float64 numpy (tolerance, FPSPEC 4).

The reference holds no golden vectors for this arithmetic (olaf_c is external,
SURVEY.md 8c) -- parity is against oracle/fp_oracle.c, which tests/test_oracle.py
pins to float64 numpy, a brute-force peak definition and known answers.
"""

import numpy as np
import pytest

import oracle as O
from aidfp import synth
from aidfp.engine import peaks_from_mask

pytestmark = pytest.mark.gpu
SR = 44100
HOP = 512


def _clip(tr, n, start=0, snr=None):
    return synth.synth(tr, start, n, SR, snr_db=snr, salt=7)


def test_power_bit_exact(gpu_engine):
    """With AID_FLAG_KEEP_POWER K1 stores every block: the power plane is the oracle's bit for bit.
    Without it (the default, `gpu_engine`) cold blocks are not stored, power() fails loudly, and
    the hashes are the same."""
    from aidfp.engine import Engine

    clips = [_clip(1, 441000), _clip(2, 100000, start=12345, snr=20), _clip(3, 2048), _clip(4, 2049), _clip(5, 5000)]
    with Engine(SR, keep_power=True) as eng:
        got_keep = eng.extract_host(clips)
        for c, x in enumerate(clips):
            P = eng.power(c, len(x))
            R = O.stft_power(x, HOP)
            assert P.shape == R.shape
            assert np.array_equal(P.view(np.uint32), R.view(np.uint32)), f"clip {c}: power bits differ"
    got = gpu_engine.extract_host(clips)
    for c in range(len(clips)):
        assert np.array_equal(got[c], got_keep[c])
    with pytest.raises(Exception, match="KEEP_POWER"):
        gpu_engine.power(0, len(clips[0]))


def test_peaks_and_hashes_bit_exact(gpu_engine):
    lens = [441000, 441000, 220500, 154350, 30000, 2047, 0, 2048 + 512 * 70]
    clips = [_clip(10 + i, n, start=777 * i, snr=20 if i % 2 else None) for i, n in enumerate(lens)]
    got = gpu_engine.extract_host(clips)
    counts = gpu_engine.counts()
    for c, x in enumerate(clips):
        ref_pk = O.peaks(O.stft_power(x, HOP)) if len(x) >= 2048 else np.zeros((0, 2), np.int32)
        pk = peaks_from_mask(gpu_engine.peakmask(c, len(x)))
        assert np.array_equal(pk, ref_pk.reshape(-1, 2)), f"clip {c}: peaks differ"
        ref = O.fingerprint(x, HOP)
        assert counts[c] == len(ref)
        assert np.array_equal(got[c], ref), f"clip {c}: hashes differ"


def test_silence_and_tiny_inputs(gpu_engine):
    clips = [np.zeros(44100, np.float32), np.zeros(0, np.float32), np.ones(100, np.float32)]
    got = gpu_engine.extract_host(clips)
    assert [len(g) for g in got] == [0, 0, 0]


def test_long_track_multi_chunk(gpu_engine):
    # 3 K3 chunks (1024 anchor frames each) and many K2 strips
    x = _clip(99, 2048 + 512 * 2600, start=5)
    got = gpu_engine.extract_host([x])[0]
    ref = O.fingerprint(x, HOP)
    assert len(ref) > 1000
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("order", ["short_first", "short_last", "short_both"])
def test_frameless_clip_beside_two_chunk_clip(gpu_engine, order):
    """A clip too short for one frame has no K3 chunk, so [short, two-chunk clip] has as many chunks as
    clips: K3 must still search the descriptors (not map chunk -> clip) and run its COUNT pass (the
    second chunk's base). Both clips' hashes equal the oracle's."""
    short = _clip(71, 1000)
    two = _clip(72, 2048 + 512 * 1500, start=99, snr=20)  # 1501 frames: 2 chunks of 1024 anchor frames
    clips = {"short_first": [short, two], "short_last": [two, short], "short_both": [short, two, short]}[order]
    got = gpu_engine.extract_host(clips)
    for c, x in enumerate(clips):
        ref = O.fingerprint(x, HOP)
        assert np.array_equal(got[c], ref), f"clip {c}: hashes differ"
    assert sum(len(g) for g in got) > 1000


def test_batch_256_full_config(gpu_engine):
    """BASELINE config 2 shape: 256 x 10 s, device-resident PCM, every clip bit-exact."""
    import torch

    n = 441000
    tracks = np.arange(1000, 1256, dtype=np.uint32)
    pcm = torch.empty(256 * n, dtype=torch.float32, device="cuda")
    gpu_engine.synth(pcm.data_ptr(), tracks, np.zeros(256, np.int64), n)
    host = pcm.cpu().numpy().reshape(256, n)
    # generator parity on a few clips
    for c in (0, 17, 255):
        assert np.array_equal(host[c], synth.synth(int(tracks[c]), 0, n, SR))
    offs = np.arange(257, dtype=np.int64) * n
    gpu_engine.extract_device(pcm.data_ptr(), offs)
    counts = gpu_engine.counts()
    ref = O.fingerprint_batch(host, HOP, threads=16)
    for c in range(256):
        assert counts[c] == len(ref[c])
        assert np.array_equal(gpu_engine.hashes(c), ref[c]), f"clip {c}"


@pytest.mark.parametrize("sr,envelope,noise", [(44100, True, 0), (44100, False, 300), (48000, True, 120),
                                               (16000, False, 0), (22050, True, 50)])
def test_synth_generators_bit_identical(gpu_engine, sr, envelope, noise):
    """aid_synth_rate (both generators, explicit rates, query noise) equals aidfp.synth bit for bit."""
    import torch

    n = sr * 2 + 5
    tracks = np.array([3, 70001, 12], np.uint32)
    starts = np.array([0, sr // 3, 7 * sr], np.int64)
    pcm = torch.empty(len(tracks) * n, dtype=torch.float32, device="cuda")
    gpu_engine.synth(pcm.data_ptr(), tracks, starts, n, noise_a=noise, salt=9, sample_rate=sr, envelope=envelope)
    host = pcm.cpu().numpy().reshape(len(tracks), n)
    for c in range(len(tracks)):
        ref = synth.synth_int16(int(tracks[c]), int(starts[c]), n, sr, noise, 9, envelope=envelope)
        assert np.array_equal(host[c], (ref.astype(np.float32) / np.float32(32768.0)).astype(np.float32)), c


def test_synth_async_two_streams(gpu_engine):
    """Two AID_SYNTH_ASYNC calls on different streams: the second call's uploads of its track and
    start arrays must not overwrite the first call's while its kernel still reads them -- both outputs equal
    the host generator."""
    import torch

    n = 44100 * 4
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    ta, sa = np.arange(40, 104, dtype=np.uint32), np.arange(64, dtype=np.int64) * 1000
    tb, sb = np.arange(900, 964, dtype=np.uint32), np.arange(64, dtype=np.int64) * 777 + 5
    a = torch.empty(64 * n, dtype=torch.float32, device="cuda")
    b = torch.empty(64 * n, dtype=torch.float32, device="cuda")
    gpu_engine.synth(a.data_ptr(), ta, sa, n, stream=s1.cuda_stream, wait=False)
    gpu_engine.synth(b.data_ptr(), tb, sb, n, stream=s2.cuda_stream, wait=False)
    s1.synchronize()
    s2.synchronize()
    ha, hb = a.cpu().numpy().reshape(64, n), b.cpu().numpy().reshape(64, n)
    for c in (0, 31, 63):
        assert np.array_equal(ha[c], synth.synth(int(ta[c]), int(sa[c]), n, SR)), c
        assert np.array_equal(hb[c], synth.synth(int(tb[c]), int(sb[c]), n, SR)), c


def test_logmag_tolerance(gpu_engine):
    """STFT magnitudes within 1e-4 rel (frame-normalised), log-mag within 60 dB of the peak."""
    x = _clip(3, 220500, snr=20)
    L = gpu_engine.spectrogram(x).astype(np.float64)
    P64 = O.stft_power_f64(x, HOP)
    L64 = 10 * np.log10(P64 + 1e-10)
    m = np.sqrt(np.maximum(10 ** (L / 10) - 1e-10, 0))
    m64 = np.sqrt(P64)
    assert (np.abs(m - m64) / m64.max(axis=1, keepdims=True)).max() <= 1e-4
    sel = P64 >= 1e-6 * P64.max(axis=1, keepdims=True)
    assert np.abs(L - L64)[sel].max() <= 1e-4 * 60.0


def test_magnitude_per_bin_1e4():
    """north_star "STFT magnitudes match within 1e-4 rel", per bin: on config-2 clips (10 s,
    44.1 kHz, synthetic v2 as the bench batch) the product path's binary32 power (K1, AID_FLAG_KEEP_POWER) gives
    magnitudes whose relative error against float64 numpy is <= 1e-4 for EVERY bin within 60 dB of its frame's
    peak (bench.magnitude_parity; the band binary32 delivers: beyond it a bin's relative error grows as it falls
    below the frame's energy, ~5e-4 at 60-80 dB). The frame-normalised test above is the secondary criterion."""
    import bench

    host = np.stack([synth.synth(int(t), 0, 441000, SR) for t in (1000, 1017, 1100, 1255)])
    r = bench.magnitude_parity(host, 4, SR)
    assert r["power_bits_equal_oracle"]
    for band in ("0-20dB", "20-40dB", "40-60dB"):
        assert r["per_bin"][band]["bins"] > 0
        assert r["per_bin"][band]["max_rel"] <= 1e-4, (band, r["per_bin"][band])
    assert r["ok"]


def test_back_to_back_calls_without_sync(gpu_engine):
    """aid_extract orders calls with events, not a stream sync per call: changed offsets,
    repeated offsets (cached descriptors), host/device PCM switches and empty clips
    queued back to back must each give the oracle's hashes."""
    import torch

    a = [_clip(40 + i, n, start=31 * i) for i, n in enumerate([44100 * 3, 30000, 44100 * 2])]
    b = [_clip(50 + i, n, start=17 * i) for i, n in enumerate([44100, 1000, 44100 * 4, 2048])]
    ref_a = [O.fingerprint(x, HOP) for x in a]
    ref_b = [O.fingerprint(x, HOP) for x in b]

    def dev(clips):
        offs = np.zeros(len(clips) + 1, np.int64)
        for i, x in enumerate(clips):
            offs[i + 1] = offs[i] + ((len(x) + 1) & ~1)
        buf = torch.zeros(int(offs[-1]), dtype=torch.float32, device="cuda")
        for i, x in enumerate(clips):
            buf[int(offs[i]):int(offs[i]) + len(x)] = torch.from_numpy(x)
        return buf, offs

    da, oa = dev(a)
    db, ob = dev(b)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(3):  # a, b, a again (cache key flips), queued without syncs
        gpu_engine.extract_device(da.data_ptr(), oa, s)
        gpu_engine.extract_device(db.data_ptr(), ob, s)
    gpu_engine.extract_device(da.data_ptr(), oa, s)
    gpu_engine.extract_device(da.data_ptr(), oa, s)  # same key twice: descriptors not re-uploaded
    got = [gpu_engine.hashes(c) for c in range(len(a))]
    for c in range(len(a)):
        assert np.array_equal(got[c], ref_a[c]), f"clip {c}"
    # host PCM with the device batch's offsets layout, then device again
    got_b = gpu_engine.extract_host(b)
    for c in range(len(b)):
        assert np.array_equal(got_b[c], ref_b[c]), f"host clip {c}"
    gpu_engine.extract_device(db.data_ptr(), ob, s)
    counts = gpu_engine.counts()
    assert counts.tolist() == [len(r) for r in ref_b]
    assert counts[1] == 0  # the 1000-sample clip has no frame


@pytest.mark.parametrize("keep", [False, True])
@pytest.mark.parametrize("hop", [128, 256, 1024, 2048])
def test_every_hop_bit_exact(hop, keep):
    """K1 is specialised per hop (hop/128 new PCM rows per frame): each specialisation is
    bit-exact, power (engine keeping the whole plane) and hashes (both store modes), including a
    long clip with several K3 chunks at hop 128."""
    from aidfp.engine import Engine

    with Engine(44100, hop=hop, keep_power=keep) as eng:
        assert eng.hop == hop
        lens = [2048, 2048 + hop * 37 + 5, 44100 * 3, 44100 * 7 + 1]
        if hop == 128:
            lens.append(2048 + 128 * 2500)  # 2501 frames: 3 K3 chunks
        clips = [_clip(70 + i, n, start=101 * i, snr=25 if i % 2 else None) for i, n in enumerate(lens)]
        got = eng.extract_host(clips)
        for c, x in enumerate(clips):
            if keep:
                P = eng.power(c, len(x))
                assert np.array_equal(P.view(np.uint32), O.stft_power(x, hop).view(np.uint32)), (hop, c)
            assert np.array_equal(got[c], O.fingerprint(x, hop)), (hop, c)


def test_max_duration_clip(gpu_engine):
    """The reference accepts uploads up to 1800 s (decode.py `decode_and_validate`
    max_duration): one 30-minute clip (155k frames, 152 K3 chunks) next to short ones."""
    long = _clip(123, SR * 1800, start=0, snr=30)
    clips = [_clip(1, 5000), long, _clip(2, SR * 5)]
    got = gpu_engine.extract_host(clips)
    for c, x in enumerate(clips):
        r = O.fingerprint(x, HOP)
        assert len(got[c]) == len(r), c
        assert np.array_equal(got[c], r), c
    assert len(got[1]) > 100000


def test_nonfinite_huge_and_tied_inputs(gpu_engine):
    """K2 compares powers as int32 keys (NaN -> 0): NaN/inf PCM (NaN and inf powers), powers that
    overflow to inf, and exactly tied powers give the oracle's peaks and hashes bit for bit."""
    rng = np.random.default_rng(3)
    a = _clip(41, 200000, snr=20)
    a[[5000, 70000, 150001]] = [np.nan, np.inf, -np.inf]
    b = _clip(42, 120000) * np.float32(3e18)  # squares overflow binary32: inf powers next to finite
    c = np.zeros(150000, np.float32)  # a repeating integer-exact pattern: tied powers across frames
    c[::512] = 8.0
    c[256::1024] = -4.0
    d = (rng.integers(-3, 4, 180000) / 4).astype(np.float32)  # coarse values, many equal powers
    clips = [a, b, c, d]
    got = gpu_engine.extract_host(clips)
    for i, x in enumerate(clips):
        ref_pk = O.peaks(O.stft_power(x, HOP))
        pk = peaks_from_mask(gpu_engine.peakmask(i, len(x)))
        assert np.array_equal(pk, ref_pk.reshape(-1, 2)), f"clip {i}: peaks differ"
        assert np.array_equal(got[i], O.fingerprint(x, HOP)), f"clip {i}: hashes differ"


def test_profile_select_masks_kernels(gpu_engine):
    """aid_profile_select: only the selected kernels get events (bench.py times K1 alone inside its
    timed region); the hashes are unchanged and `None` restores every kernel."""
    clips = [_clip(70 + i, 44100 * 2 + 512 * i) for i in range(3)]
    ref = [O.fingerprint(x, HOP) for x in clips]
    try:
        gpu_engine.profile_select([0])
        gpu_engine.profile_enable(True)
        gpu_engine.profile_read(reset=True)
        got = gpu_engine.extract_host(clips)
        prof = gpu_engine.profile_read(reset=True)
        assert prof["stft_power"][1] == 1 and prof["stft_power"][0] > 0
        assert all(cnt == 0 for k, (_, cnt) in prof.items() if k != "stft_power")
        for g, r in zip(got, ref):
            assert np.array_equal(g, r)
        gpu_engine.profile_select(None)
        gpu_engine.extract_host(clips)
        prof = gpu_engine.profile_read(reset=True)
        assert prof["stft_power"][1] == 1 and prof["peak_pick"][1] == 1
    finally:
        gpu_engine.profile_enable(False)
        gpu_engine.profile_select(None)
        gpu_engine.profile_read(reset=True)


def test_band_limited_quarters_bit_exact(gpu_engine):
    """Content confined to one or two bands, with tones on the 64-bin block and 256-bin quarter
    edges: K2's per-wave strip-cold skip (a quarter whose +-1-block window is cold in every row of
    the strip writes zero mask words without running the row loop) is taken by different waves in
    different clips, and the hot quarters' +-15-bin windows straddle the skipped ones."""
    rng = np.random.default_rng(5)
    n = 44100 * 3
    t = np.arange(n) / SR
    clips = []
    for bins in ([10], [250, 262], [511, 513], [700], [767, 769, 1000], [60, 1010], [383, 384, 449]):
        x = np.zeros(n)
        for k in bins:
            f = k * SR / 2048.0
            am = 0.5 + 0.5 * np.sin(2 * np.pi * rng.uniform(1, 4) * t + rng.uniform(0, 6))
            x += 0.05 * am * np.sin(2 * np.pi * f * t + rng.uniform(0, 6))
        x += rng.standard_normal(n) * 1e-4
        clips.append(np.clip(x, -1, 1).astype(np.float32))
    got = gpu_engine.extract_host(clips)
    for c, x in enumerate(clips):
        ref_pk = O.peaks(O.stft_power(x, HOP))
        pk = peaks_from_mask(gpu_engine.peakmask(c, len(x)))
        assert np.array_equal(pk, ref_pk.reshape(-1, 2)), f"clip {c}: peaks differ"
        ref = O.fingerprint(x, HOP)
        assert len(ref) > 0
        assert np.array_equal(got[c], ref), f"clip {c}: hashes differ"


@pytest.mark.parametrize("slots_x", ["1", "1.25", "1.5", "3"])
def test_k2_strip_multipliers_bit_exact(slots_x):
    """K2's strip count follows the measured cold-wave fraction (1, 1.25 or 1.5 strips per resident
    workgroup slot, engine.cpp extract_locked; strip-cold waves exit). Every fixed multiplier, including
    one that leaves workgroups waiting for slots, gives the oracle's peaks and hashes bit for bit, on a
    band-limited batch where about half of the quarter waves are strip-cold and exit."""
    from aidfp.engine import Engine

    clips = [_clip(t, 44100 * 4 + 313 * t, snr=None if t % 3 else 20) for t in range(24)]
    with Engine(SR) as eng:
        eng.force("k2_strips_x100", round(float(slots_x) * 100))
        got = eng.extract_host(clips)
        for c, x in enumerate(clips):
            pk = peaks_from_mask(eng.peakmask(c, len(x)))
            assert np.array_equal(pk, O.peaks(O.stft_power(x, HOP)).reshape(-1, 2)), f"clip {c}: peaks differ"
            assert np.array_equal(got[c], O.fingerprint(x, HOP)), f"clip {c}: hashes differ"


@pytest.mark.parametrize("rows", [0, 1, 700, 2000])
def test_clip_groups_bit_exact(rows):
    """A call whose frames exceed the plane bound runs K1 -> K2 per group of clips on one power buffer (engine.cpp
    extract_locked, kPlaneRows; `plane_rows` forces the bound). Every grouping gives the oracle's peaks and hashes:
    a group per clip (1), several clips per group with a clip longer than the bound alone in its group (700, 2000
    rows; the 40 s clip has 3,445 frames), and one group (0); host and device PCM, and calls repeated (cached
    descriptors keyed on the groups)."""
    import torch

    from aidfp.engine import Engine

    lens = [44100 * 4 + 313 * t for t in range(9)] + [44100 * 40, 100, 44100 * 3]
    clips = [_clip(t, n, snr=None if t % 3 else 20) for t, n in enumerate(lens)]
    refs = [O.fingerprint(x, HOP) for x in clips]
    with Engine(SR) as eng:
        eng.force("plane_rows", rows)
        for _ in range(2):
            got = eng.extract_host(clips)
            for c, x in enumerate(clips):
                pk = peaks_from_mask(eng.peakmask(c, len(x)))
                assert np.array_equal(pk, O.peaks(O.stft_power(x, HOP)).reshape(-1, 2)), f"clip {c}: peaks differ"
                assert np.array_equal(got[c], refs[c]), f"clip {c}: hashes differ"
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        dev = torch.from_numpy(np.concatenate(clips).astype(np.float32)).cuda()
        eng.extract_device(dev.data_ptr(), offs)
        for c in range(len(clips)):
            assert np.array_equal(eng.hashes(c), refs[c]), f"device PCM, clip {c}: hashes differ"
