"""Python face of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline. It never backs the
product path (audio-ident_amd/aidfp -> libaidfp.so, HIP on gfx950).

Two oracles live here:
  * ``fp_*`` -- ctypes over ``_build/libfporacle.so`` (fp_oracle.c / fp_match.c):
    the binary32 restatement of spec/FPSPEC.md, bit-exact target for the GPU.
  * ``stft_power_f64`` / ``logmag_f64`` -- numpy float64 rfft (pocketfft) of the
    same frames: the independent accuracy reference (tolerance, not bits).

Parity status: the reference's fingerprint arithmetic lives in the external
``olaf_c`` binary (audio-ident-service/app/audio/fingerprint.py:117-125,
185-193) which is absent from /root/reference, so hash parity is **unpinned by
the reference**; this oracle is pinned by float64 numpy, a brute-force peak
definition and known-answer tests (tests/test_oracle.py).
"""

from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "_build" / "libfporacle.so"
N_FFT = 2048
BINS = 1024
DEFAULT_THR = 4.0


def build() -> Path:
    srcs = [HERE / "fp_oracle.c", HERE / "fp_match.c", HERE / "fp_resample.c", HERE / "fp_dedup.c"]
    if not LIB_PATH.exists() or any(s.stat().st_mtime > LIB_PATH.stat().st_mtime for s in srcs):
        subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


_lib = None


class Posting(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_uint32), ("track", ctypes.c_uint32), ("t", ctypes.c_uint32)]


class Row(ctypes.Structure):
    _fields_ = [
        ("match_count", ctypes.c_int32),
        ("track", ctypes.c_uint32),
        ("d", ctypes.c_int32),
        ("tq_min", ctypes.c_int32),
        ("tq_max", ctypes.c_int32),
    ]


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        L.fp_num_frames.restype = i64
        L.fp_num_frames.argtypes = [i64, ctypes.c_int]
        L.fp_stft_power.restype = i64
        L.fp_stft_power.argtypes = [P, i64, ctypes.c_int, P]
        for name in ("fp_peaks", "fp_peaks_bruteforce"):
            f = getattr(L, name)
            f.restype = i64
            f.argtypes = [P, i64, ctypes.c_float, P, P, i64]
        L.fp_hashes.restype = i64
        L.fp_hashes.argtypes = [P, P, i64, P, P, i64]
        L.fp_peak_capacity.restype = i64
        L.fp_peak_capacity.argtypes = [i64]
        L.fp_fingerprint.restype = i64
        L.fp_fingerprint.argtypes = [P, i64, ctypes.c_int, ctypes.c_float, P, P, i64]
        L.fp_fingerprint_batch.restype = ctypes.c_int
        L.fp_fingerprint_batch.argtypes = [P, i64, ctypes.c_int, ctypes.c_int, ctypes.c_float, P, P, i64, P, ctypes.c_int]
        L.fp_index_sort.restype = None
        L.fp_index_sort.argtypes = [P, i64]
        L.fp_query.restype = i64
        L.fp_query.argtypes = [P, i64, P, P, i64, ctypes.c_int32, P, i64]
        L.fp_resample_ratio.argtypes = [ctypes.c_int32] * 2 + [P] * 4
        L.fp_resample_taps.argtypes = [ctypes.c_int32, ctypes.c_int32, P]
        L.fp_resample_len.restype = i64
        L.fp_resample_len.argtypes = [i64, ctypes.c_int32, ctypes.c_int32]
        L.fp_resample.restype = i64
        L.fp_resample.argtypes = [P, i64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, P]
        L.fp_dedup_similarity.restype = ctypes.c_double
        L.fp_dedup_similarity.argtypes = [P, i64, P, i64]
        L.fp_dedup_scan.argtypes = [P, P, P, i64, P, P, P, i64, P, P]
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data)


def num_frames(n: int, hop: int) -> int:
    return 0 if n < N_FFT else 1 + (n - N_FFT) // hop


def default_hop(sr: int) -> int:
    return 512 if sr >= 32000 else 256


def stft_power(x: np.ndarray, hop: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    F = num_frames(len(x), hop)
    P = np.zeros((F, BINS), dtype=np.float32)
    if F:
        lib().fp_stft_power(_ptr(x), len(x), hop, _ptr(P))
    return P


def peaks(P: np.ndarray, thr: float = DEFAULT_THR, brute: bool = False) -> np.ndarray:
    """[n, 2] int32 (t, k) in (t, k) order."""
    P = np.ascontiguousarray(P, dtype=np.float32)
    F = P.shape[0]
    cap = max(1, int(lib().fp_peak_capacity(F)))
    pt = np.zeros(cap, dtype=np.int32)
    pk = np.zeros(cap, dtype=np.int32)
    f = lib().fp_peaks_bruteforce if brute else lib().fp_peaks
    n = int(f(_ptr(P), F, thr, _ptr(pt), _ptr(pk), cap))
    assert n <= cap, "peak packing bound violated"
    return np.stack([pt[:n], pk[:n]], axis=1)


def hashes_from_peaks(pk: np.ndarray) -> np.ndarray:
    """[n] uint64 records: hash | t1 << 32."""
    pk = np.ascontiguousarray(pk, dtype=np.int32)
    t = np.ascontiguousarray(pk[:, 0])
    k = np.ascontiguousarray(pk[:, 1])
    cap = max(1, 10 * len(t))
    h = np.zeros(cap, dtype=np.uint32)
    t1 = np.zeros(cap, dtype=np.uint32)
    n = int(lib().fp_hashes(_ptr(t), _ptr(k), len(t), _ptr(h), _ptr(t1), cap))
    return h[:n].astype(np.uint64) | (t1[:n].astype(np.uint64) << np.uint64(32))


def fingerprint(x: np.ndarray, hop: int, thr: float = DEFAULT_THR) -> np.ndarray:
    """Whole pipeline for one clip -> [n] uint64 records (hash | t1 << 32)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    F = num_frames(len(x), hop)
    cap = max(1, 10 * int(lib().fp_peak_capacity(F)))
    h = np.zeros(cap, dtype=np.uint32)
    t1 = np.zeros(cap, dtype=np.uint32)
    n = int(lib().fp_fingerprint(_ptr(x), len(x), hop, thr, _ptr(h), _ptr(t1), cap))
    if n < 0:
        raise MemoryError("oracle allocation failed")
    return h[:n].astype(np.uint64) | (t1[:n].astype(np.uint64) << np.uint64(32))


def fingerprint_batch(x: np.ndarray, hop: int, thr: float = DEFAULT_THR, threads: int = 1):
    """[C, n] batch -> (list of per-clip uint64 record arrays)."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    C, n = x.shape
    F = num_frames(n, hop)
    cap = max(1, 10 * int(lib().fp_peak_capacity(F)))
    h = np.zeros((C, cap), dtype=np.uint32)
    t1 = np.zeros((C, cap), dtype=np.uint32)
    counts = np.zeros(C, dtype=np.int64)
    lib().fp_fingerprint_batch(_ptr(x), n, C, hop, thr, _ptr(h), _ptr(t1), cap, _ptr(counts), threads)
    return [h[c, : counts[c]].astype(np.uint64) | (t1[c, : counts[c]].astype(np.uint64) << np.uint64(32)) for c in range(C)]


def query(postings: np.ndarray, q_records: np.ndarray, min_match: int = 5, max_rows: int = 50) -> np.ndarray:
    """postings: structured/uint32 [n,3] (hash, track, t); q_records: uint64 (hash | t << 32).

    Returns [r, 5] int64 rows (match_count, track, d, tq_min, tq_max)."""
    p = np.ascontiguousarray(postings, dtype=np.uint32).reshape(-1, 3).copy()
    lib().fp_index_sort(_ptr(p), len(p))
    q = np.ascontiguousarray(q_records, dtype=np.uint64)
    qh = np.ascontiguousarray((q & np.uint64(0xFFFFFFFF)).astype(np.uint32))
    qt = np.ascontiguousarray((q >> np.uint64(32)).astype(np.uint32))
    rows = (Row * max(1, max_rows))()
    n = int(lib().fp_query(_ptr(p), len(p), _ptr(qh), _ptr(qt), len(q), min_match, ctypes.addressof(rows), max_rows))
    return np.array([[r.match_count, r.track, r.d, r.tq_min, r.tq_max] for r in rows[:n]], dtype=np.int64).reshape(-1, 5)


# ---- float64 numpy reference (accuracy, not bits) ----

def frames_f64(x: np.ndarray, hop: int) -> np.ndarray:
    x = np.asarray(x, dtype=np.float64)
    F = num_frames(len(x), hop)
    if F == 0:
        return np.zeros((0, N_FFT))
    idx = np.arange(F)[:, None] * hop + np.arange(N_FFT)[None, :]
    return x[idx]


def window_f64() -> np.ndarray:
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(N_FFT) / N_FFT)


def stft_power_f64(x: np.ndarray, hop: int) -> np.ndarray:
    fr = frames_f64(x, hop) * window_f64()[None, :]
    X = np.fft.rfft(fr, axis=1)[:, :BINS]
    return X.real**2 + X.imag**2


def logmag_f64(x: np.ndarray, hop: int) -> np.ndarray:
    return 10.0 * np.log10(stft_power_f64(x, hop) + 1e-10)


# ---------------------------------------------------------------- NumPy/SciPy CPU path (timing baseline)

def fingerprint_numpy(x: np.ndarray, hop: int, thr: float = DEFAULT_THR) -> np.ndarray:
    """FPSPEC 4-6 written the way a NumPy/SciPy user would (BASELINE north_star: "the reference
    NumPy/SciPy CPU path"; the reference itself has none): framed float64 rfft
    (pocketfft), scipy.ndimage.maximum_filter over the 15 x 31 neighbourhood with the earliest-wins
    tie rule applied to the few tied maxima, vectorised anchor/target pairing. It is the bench's
    cpu_baseline "numpy_scipy" leg only: float64 arithmetic, so its records are not bit-exact with
    the binary32 spec (fp_oracle.c is the checker); `tests/test_oracle.py` bounds the difference."""
    from scipy.ndimage import maximum_filter

    P = stft_power_f64(x, hop)
    F = P.shape[0]
    if F == 0:
        return np.zeros(0, dtype=np.uint64)
    mx = maximum_filter(P, size=(15, 31), mode="constant", cval=-1.0)
    cand = (P == mx) & (P > thr)
    cand[:, 0] = False
    # ties: of two candidates in each other's neighbourhood (equal maxima) the later in (t, k) order loses
    from scipy.ndimage import uniform_filter

    crowd = uniform_filter(cand.astype(np.float64), size=(15, 31), mode="constant") * (15 * 31) > 1.5
    t, k = np.nonzero(cand)  # (t, k) order
    tied = np.nonzero(crowd[t, k])[0]
    if len(tied) > 1:
        keep = np.ones(len(t), dtype=bool)
        for a_, i in enumerate(tied):
            if not keep[i]:
                continue
            o = tied[a_ + 1:]
            near = (np.abs(t[o] - t[i]) <= 7) & (np.abs(k[o] - k[i]) <= 15)
            keep[o[near]] = False
        t, k = t[keep], k[keep]
    n = len(t)
    if n < 2:
        return np.zeros(0, dtype=np.uint64)
    # pairing: anchor i with the peaks i+1 .. i+D in order (the target zone spans < 64 frames)
    D = int(min(n - 1, 64 * 64))
    out_h, out_t, out_i, out_j = [], [], [], []
    taken = np.zeros(n, dtype=np.int64)
    for d in range(1, D + 1):
        i = np.arange(n - d)
        j = i + d
        dt = t[j] - t[i]
        if dt.min() > 63:
            break
        ok = (dt > 0) & (dt <= 63) & (np.abs(k[j] - k[i]) <= 127) & (taken[i] < 10)
        taken[i[ok]] += 1
        ii, jj = i[ok], j[ok]
        out_h.append((k[ii].astype(np.uint64) << 22) | (k[jj].astype(np.uint64) << 12) | (t[jj] - t[ii]).astype(np.uint64))
        out_t.append(t[ii].astype(np.uint64))
        out_i.append(ii)
        out_j.append(jj)
    if not out_h:
        return np.zeros(0, dtype=np.uint64)
    h, ta, ai, aj = (np.concatenate(v) for v in (out_h, out_t, out_i, out_j))
    order = np.lexsort((aj, ai))  # anchor, then target order
    return h[order] | (ta[order] << np.uint64(32))


if os.environ.get("AIDFP_ORACLE_AUTOBUILD", "1") == "1" and not LIB_PATH.exists():
    try:
        build()
    except Exception:  # pragma: no cover - surfaced by lib()
        pass


# ---- PCM front-end (FPSPEC 8): downmix + rational resampling ----
def resample_ratio(sr_in: int, sr_out: int):
    v = [ctypes.c_int32() for _ in range(4)]
    if not lib().fp_resample_ratio(sr_in, sr_out, *[ctypes.byref(x) for x in v]):
        raise ValueError("bad sample rates")
    return tuple(x.value for x in v)  # up, down, hl, J


def resample_taps(sr_in: int, sr_out: int) -> np.ndarray:
    up, down, hl, _ = resample_ratio(sr_in, sr_out)
    t = np.zeros(2 * hl + 1, np.float32)
    lib().fp_resample_taps(up, down, _ptr(t))
    return t


def resample(x: np.ndarray, sr_in: int, sr_out: int) -> np.ndarray:
    """x: [n] mono or [n, 2] interleaved stereo float32 -> mono float32 at sr_out."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    ch = 1 if x.ndim == 1 else x.shape[1]
    n = x.shape[0]
    y = np.zeros(max(1, int(lib().fp_resample_len(n, sr_in, sr_out))), np.float32)
    m = lib().fp_resample(_ptr(x), n, ch, sr_in, sr_out, _ptr(y))
    return y[:m]


# ---- Chromaprint dedup scan (dedup.py:127-222) ----
def _pack_u32(arrs):
    off = np.zeros(len(arrs) + 1, dtype=np.int64)
    if arrs:
        off[1:] = np.cumsum([len(a) for a in arrs])
    w = np.concatenate(arrs).astype(np.uint32) if arrs and off[-1] else np.zeros(1, np.uint32)
    return np.ascontiguousarray(w), off


def dedup_scan(cat, cat_dur, queries, q_dur):
    """cat/queries: lists of uint32 arrays. Returns (best_idx int64[nq] (-1 = none), best_sim f64[nq])."""
    cw, co = _pack_u32(cat)
    qw, qo = _pack_u32(queries)
    cd = np.ascontiguousarray(cat_dur, dtype=np.float64)
    qd = np.ascontiguousarray(q_dur, dtype=np.float64)
    nq = len(queries)
    bi = np.zeros(max(1, nq), np.int64)
    bs = np.zeros(max(1, nq), np.float64)
    lib().fp_dedup_scan(_ptr(cw), _ptr(co), _ptr(cd), len(cat), _ptr(qw), _ptr(qo), _ptr(qd), nq, _ptr(bi), _ptr(bs))
    return bi[:nq], bs[:nq]
