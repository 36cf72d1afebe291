"""Python handle on one libaidfp engine (one GPU).

Thin: it marshals numpy arrays / raw device pointers into the C ABI of
include/aidfp.h. Device memory for benchmark inputs comes from torch (plumbing
only); nothing here computes a fingerprint itself.
"""

from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from . import _lib as L
from ._lib import AID_ERR_DEVICE, AID_PCM_DEVICE, AID_PCM_HOST, AidConfig, EngineError, EngineUnavailable, check

N_FFT = 2048
BINS = 1024


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


class Engine:
    def __init__(self, sample_rate: int, hop: int = 0, peak_threshold: float = 0.0, device: int = -1,
                 min_match: int = 0, max_results: int = 0):
        lib = L.load()
        cfg = AidConfig()
        check(lib.aid_config_default(int(sample_rate), ctypes.byref(cfg)))
        if hop:
            cfg.hop = hop
        if peak_threshold:
            cfg.peak_threshold = peak_threshold
        cfg.device = device
        if min_match:
            cfg.min_match = min_match
        if max_results:
            cfg.max_results = max_results
        h = ctypes.c_void_p()
        rc = lib.aid_engine_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc == AID_ERR_DEVICE:
            raise EngineUnavailable(L.last_error())
        check(rc)
        self._h = h
        self._lib = lib
        out = AidConfig()
        check(lib.aid_engine_config(h, ctypes.byref(out)))
        self.sample_rate = out.sample_rate
        self.hop = out.hop
        self.peak_threshold = out.peak_threshold
        self.device = out.device
        self.min_match = out.min_match
        self.max_results = out.max_results
        self.n_clips = 0

    # -- lifecycle --
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.aid_engine_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- sizes --
    def num_frames(self, n: int) -> int:
        return int(self._lib.aid_num_frames(self._h, int(n)))

    def hash_capacity(self, n: int) -> int:
        return int(self._lib.aid_hash_capacity(self._h, int(n)))

    # -- extraction --
    def extract_host(self, clips: Sequence[np.ndarray]) -> list[np.ndarray]:
        """Fingerprint host clips; returns one uint64 record array (hash | t1 << 32) per clip."""
        arrs = [np.ascontiguousarray(c, dtype=np.float32).ravel() for c in clips]
        offsets = np.zeros(len(arrs) + 1, dtype=np.int64)
        if arrs:
            offsets[1:] = np.cumsum([len(a) for a in arrs])
        pcm = np.concatenate(arrs) if arrs else np.zeros(1, dtype=np.float32)
        if pcm.size == 0:
            pcm = np.zeros(1, dtype=np.float32)
        check(self._lib.aid_extract(self._h, _p(pcm), _p(offsets), len(arrs), AID_PCM_HOST, None))
        self.n_clips = len(arrs)
        return [self.hashes(c) for c in range(len(arrs))]

    def extract_device(self, pcm_ptr: int, offsets: np.ndarray, stream: int | None = None) -> None:
        """Asynchronous extraction of device PCM; offsets = host int64[n_clips+1] (even)."""
        offsets = np.ascontiguousarray(offsets, dtype=np.int64)
        check(self._lib.aid_extract(self._h, ctypes.c_void_p(pcm_ptr), _p(offsets), len(offsets) - 1,
                                    AID_PCM_DEVICE, ctypes.c_void_p(stream) if stream else None))
        self.n_clips = len(offsets) - 1

    def sync(self) -> None:
        check(self._lib.aid_sync(self._h))

    def counts(self) -> np.ndarray:
        out = np.zeros(max(1, self.n_clips), dtype=np.int64)
        check(self._lib.aid_result_counts(self._h, _p(out)))
        return out[: self.n_clips]

    def hashes(self, clip: int) -> np.ndarray:
        n = ctypes.c_int64(0)
        rc = self._lib.aid_result_hashes(self._h, clip, None, 0, ctypes.byref(n))
        if rc != 0 and n.value == 0:
            check(rc)
        out = np.zeros(max(1, n.value), dtype=np.uint64)
        check(self._lib.aid_result_hashes(self._h, clip, _p(out), n.value, ctypes.byref(n)))
        return out[: n.value]

    def device_view(self):
        """(records_ptr, counts_dev_ptr, clip_base np.int64[n_clips]) of the last extraction."""
        rec = ctypes.c_void_p()
        cnt = ctypes.c_void_p()
        base = ctypes.POINTER(ctypes.c_int64)()
        n = ctypes.c_int32()
        check(self._lib.aid_result_device(self._h, ctypes.byref(rec), ctypes.byref(cnt), ctypes.byref(base),
                                          ctypes.byref(n)))
        bases = np.ctypeslib.as_array(base, shape=(n.value,)).copy() if n.value else np.zeros(0, np.int64)
        return rec.value, cnt.value, bases

    def power(self, clip: int, n_samples: int) -> np.ndarray:
        F = self.num_frames(n_samples)
        out = np.zeros((max(F, 1), BINS), dtype=np.float32)
        check(self._lib.aid_result_power(self._h, clip, _p(out), out.size))
        return out[:F]

    def peakmask(self, clip: int, n_samples: int) -> np.ndarray:
        F = self.num_frames(n_samples)
        out = np.zeros((max(F, 1), 16), dtype=np.uint64)
        check(self._lib.aid_result_peakmask(self._h, clip, _p(out), out.size))
        return out[:F]

    def spectrogram(self, x: np.ndarray) -> np.ndarray:
        """GPU log-magnitude 10*log10(P + 1e-10), [F, 1024]."""
        x = np.ascontiguousarray(x, dtype=np.float32)
        F = self.num_frames(len(x))
        out = np.zeros((max(F, 1), BINS), dtype=np.float32)
        check(self._lib.aid_spectrogram(self._h, _p(x), len(x), _p(out), out.size))
        return out[:F]

    def synth(self, dst_ptr: int, tracks, starts, n: int, noise_a: int = 0, salt: int = 0,
              stream: int | None = None) -> None:
        tr = np.ascontiguousarray(tracks, dtype=np.uint32)
        st = np.ascontiguousarray(starts, dtype=np.int64)
        check(self._lib.aid_synth(self._h, ctypes.c_void_p(dst_ptr), _p(tr), _p(st), len(tr), int(n), int(noise_a),
                                  int(salt) & 0xFFFFFFFF, ctypes.c_void_p(stream) if stream else None))

    # -- profiling --
    def profile_enable(self, on: bool = True) -> None:
        check(self._lib.aid_profile_enable(self._h, 1 if on else 0))

    def profile_read(self, reset: bool = False) -> dict:
        ms = np.zeros(L.AID_K_COUNT, dtype=np.float64)
        n = np.zeros(L.AID_K_COUNT, dtype=np.int64)
        check(self._lib.aid_profile_read(self._h, _p(ms), _p(n), 1 if reset else 0))
        return {name: (float(ms[i]), int(n[i])) for i, name in enumerate(L.KERNEL_NAMES)}


def peaks_from_mask(mask: np.ndarray) -> np.ndarray:
    """[F,16] uint64 K2 mask -> [n,2] int32 (t, k) in (t, k) order.

    K2's ballot layout: word 4*w + i, bit l = peak flag of bin 256*w + 4*l + i."""
    F = mask.shape[0]
    bits = np.unpackbits(mask.astype("<u8").view(np.uint8).reshape(F, 16, 8), axis=2, bitorder="little")
    bits = bits.reshape(F, 4, 4, 64)  # [F][w][i][l]
    nat = bits.transpose(0, 1, 3, 2).reshape(F, 1024)  # bin = 256w + 4l + i
    t, k = np.nonzero(nat)
    return np.stack([t, k], axis=1).astype(np.int32)


__all__ = ["Engine", "EngineError", "EngineUnavailable", "peaks_from_mask"]
