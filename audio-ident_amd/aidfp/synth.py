"""Deterministic synthetic PCM, integer-exact.

Every sample is computed with uint32/int32 integer arithmetic and quantised to
int16 before the single exact division by 32768, so this numpy version, the C
oracle tests and the GPU kernel ``aid_synth`` (csrc/synth.hip) produce
bit-identical float32 PCM.

Semantics follow the reference's evaluation corpus builder: seed 42
(``audio-ident-service/scripts/build_eval_corpus.py:48-51``), white-noise
variants at a target SNR in dB (``build_eval_corpus.py:154-198``, default 20 dB
at ``:602-606``) and query offsets drawn uniformly (``:481-483``).

Signal of track ``tr`` at absolute sample ``i``:
  * 8 partials ``p``: phase increment ``inc = inc_min + (R(tr,p,j) * inc_rng) >> 32``
    (100 Hz .. 8 kHz; ``fmax_hz`` widens the band, e.g. 20 kHz for the full-band workload), amplitude
    ``A = 983 + R(tr,p+8,j) % 2949`` (0.03 .. 0.12 FS), phase ``ph = R(tr,p+16,j) + inc * rel`` (mod 2^32),
    value ``(A' * SIN[ph >> 20]) >> 15`` with ``SIN[k] = round(32767 sin(2 pi k / 4096))``, where ``j`` is the
    partial's note index and ``rel`` the sample's offset in that note:
      - generator v2 (default, ``envelope=True``): every track has its own tempo,
        ``note_len = ((sr // 4) * (12 + R(tr,40,0) % 9)) // 16`` (0.19 .. 0.31 s), every partial its own
        onset phase ``off = (note_len * (R(tr,p+32,0) % 1024)) // 1024`` (``j = (i + off) // note_len``), and
        every note decays linearly to half amplitude, ``A' = (A * E) >> 16`` with
        ``E = 65536 - (rel * 32768) // note_len``, as a struck or plucked note: landmark times lock to the
        onsets, and the instruments' independent rhythms give the landmark pairs their spread of dt;
      - generator v0 (``envelope=False``): one grid for every track and partial, ``note_len = sr // 4``
        (250 ms), ``j = i // note_len``, ``A' = A`` (stationary notes). On a stationary note the peak frame is
        decided by noise, so an independent capture of the same track (another rate, another noise floor)
        kept only ~2 % of the landmarks; v0 remains for the oracle's golden fixture;
  * base noise ``R(tr,24,i) % 1137 - 568`` (about -40 dBFS rms);
  * optional query noise ``R(tr ^ salt, 25, i) % (2a+1) - a`` (``a`` from the SNR);
  * sum, clip to int16, divide by 32768.
"""

from __future__ import annotations

import numpy as np

SEED = 42
N_PARTIALS = 8
_SIN_TABLE = np.round(32767.0 * np.sin(2.0 * np.pi * np.arange(4096) / 4096.0)).astype(np.int64)
# nominal signal rms in int16 units: 8 partials, mean amplitude 2457.5, rms A/sqrt(2)
NOMINAL_RMS = float(np.sqrt(N_PARTIALS * (2457.5**2) / 2.0))


def sin_table() -> np.ndarray:
    return _SIN_TABLE.astype(np.int16)


def _mix(x: np.ndarray) -> np.ndarray:
    """lowbias32 integer hash on uint32 arrays."""
    x = x.astype(np.uint32, copy=True)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def rnd(track, stream, idx) -> np.ndarray:
    """R(track, stream, idx) = mix(mix(mix(track + SEED*0x9E3779B9) + stream*0x85EBCA6B) + idx)."""
    with np.errstate(over="ignore"):
        t = np.asarray(track, dtype=np.uint32)
        a = _mix(t + np.uint32((SEED * 0x9E3779B9) & 0xFFFFFFFF))
        b = _mix(a + np.uint32((int(stream) * 0x85EBCA6B) & 0xFFFFFFFF))
        return _mix(b + np.asarray(idx, dtype=np.uint64).astype(np.uint32))


def inc_params(sr: int, fmax_hz: int = 8000) -> tuple[int, int]:
    inc_min = int(np.floor(100.0 / sr * 4294967296.0))
    inc_rng = int(np.floor((fmax_hz - 100) / sr * 4294967296.0))
    return inc_min, inc_rng


def noise_halfwidth(snr_db: float | None) -> int:
    """Half-width (int16 units) of uniform noise giving ``snr_db`` vs NOMINAL_RMS; 0 = none."""
    if snr_db is None:
        return 0
    rms = NOMINAL_RMS / (10.0 ** (snr_db / 20.0))
    return int(round(rms * np.sqrt(3.0)))


def note_params(track: int, sr: int, envelope: bool = True) -> tuple[int, list[int]]:
    """(note_len, per-partial onset offsets) of a track (generator v2; v0: sr // 4 and zeros)."""
    if not envelope:
        return sr // 4, [0] * N_PARTIALS
    note_len = ((sr // 4) * (12 + int(rnd(track, 40, 0)) % 9)) // 16
    return note_len, [(note_len * (int(rnd(track, p + 32, 0)) % 1024)) // 1024 for p in range(N_PARTIALS)]


def synth_int16(track: int, start: int, n: int, sr: int, noise_a: int = 0, salt: int = 0,
                fmax_hz: int = 8000, envelope: bool = True) -> np.ndarray:
    """int32 array of int16-range samples of track ``track`` at absolute samples start..start+n."""
    if n <= 0:
        return np.zeros(0, dtype=np.int32)
    note_len, offs = note_params(track, sr, envelope)
    inc_min, inc_rng = inc_params(sr, fmax_hz)
    i = np.arange(start, start + n, dtype=np.int64)
    acc = np.zeros(n, dtype=np.int64)
    with np.errstate(over="ignore"):
        for p in range(N_PARTIALS):
            ip = i + offs[p]
            j = ip // note_len
            rel = (ip - j * note_len).astype(np.uint64)
            r = rnd(track, p, j).astype(np.uint64)
            inc = (np.uint64(inc_min) + ((r * np.uint64(inc_rng)) >> np.uint64(32))) & np.uint64(0xFFFFFFFF)
            amp = 983 + (rnd(track, p + 8, j).astype(np.int64) % 2949)
            if envelope:
                amp = (amp * (65536 - (rel.astype(np.int64) * 32768) // note_len)) >> 16
            ph = (rnd(track, p + 16, j).astype(np.uint64) + inc * rel) & np.uint64(0xFFFFFFFF)
            acc += (amp * _SIN_TABLE[(ph >> np.uint64(20)).astype(np.int64)]) >> 15
        acc += rnd(track, 24, i).astype(np.int64) % 1137 - 568
        if noise_a > 0:
            acc += rnd(np.uint32(track) ^ np.uint32(salt), 25, i).astype(np.int64) % (2 * noise_a + 1) - noise_a
    return np.clip(acc, -32768, 32767).astype(np.int32)


def synth(track: int, start: int, n: int, sr: int, snr_db: float | None = None, salt: int = 0,
          fmax_hz: int = 8000, envelope: bool = True) -> np.ndarray:
    """float32 PCM in [-1, 1): int16 samples / 32768 (exact)."""
    q = synth_int16(track, start, n, sr, noise_halfwidth(snr_db), salt, fmax_hz, envelope)
    return (q.astype(np.float32) / np.float32(32768.0)).astype(np.float32)


def synth_batch(tracks, n: int, sr: int, starts=None, snr_db: float | None = None, salt: int = 0) -> np.ndarray:
    """[len(tracks), n] float32 batch."""
    tracks = list(tracks)
    starts = [0] * len(tracks) if starts is None else list(starts)
    out = np.empty((len(tracks), n), dtype=np.float32)
    for c, (tr, st) in enumerate(zip(tracks, starts)):
        out[c] = synth(int(tr), int(st), n, sr, snr_db, salt)
    return out
