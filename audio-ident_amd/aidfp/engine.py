"""Python handle on one libaidfp engine (one GPU).

Thin: it marshals numpy arrays / raw device pointers into the C ABI of
include/aidfp.h. Device memory for benchmark inputs comes from torch (plumbing
only); nothing here computes a fingerprint itself.
"""

from __future__ import annotations

import atexit
import ctypes
import os
import sys
import threading
import weakref
from typing import Sequence

import numpy as np

from . import _lib as L
from ._lib import (AID_ERR_DEVICE, AID_PCM_DEVICE, AID_PCM_HOST, AidConfig, EngineError,
                   EngineUnavailable, check)

N_FFT = 2048
BINS = 1024


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


class _PinnedSlot:
    """One thread's page-locked staging buffer (a thread's slot dies with the thread)."""

    __slots__ = ("buf", "__weakref__")

    def __init__(self):
        self.buf = None


_pinned = threading.local()
_PINNED_MAX = 16 << 20  # floats (64 MiB: the query coalescer's batch cap); larger host batches stay pageable

# Ordered teardown. Everything that owns device or page-locked memory is released from ONE atexit hook, registered
# after torch's own (atexit runs last-registered first), so it runs while the HIP runtime, torch's allocators and
# any profiler tool (rocprofv3) are all still alive: the live engines are destroyed, the service threads joined,
# every thread's page-locked staging buffer dropped and torch's pinned cache emptied. Afterwards Engine.__del__ is
# a no-op, so nothing calls into HIP while the interpreter or the C runtime tears down.
_live: "weakref.WeakSet[Engine]" = weakref.WeakSet()
_pinned_slots: "weakref.WeakSet[_PinnedSlot]" = weakref.WeakSet()  # every live thread's staging slot
_closers: "weakref.WeakSet" = weakref.WeakSet()  # objects closed first (FingerprintService: its threads, its engine)
_shutdown_done = False
_hook_lock = threading.Lock()
_hook_registered = False


def _finalizing() -> bool:
    return _shutdown_done or sys.is_finalizing()


def on_shutdown(obj) -> None:
    """obj.close() runs in the ordered teardown before the engines are destroyed (a service joins its threads
    first). Held weakly: an object that is gone by then has nothing left to close."""
    _register_hook()
    _closers.add(obj)


def _shutdown() -> None:
    global _shutdown_done, _copy_pool
    if _shutdown_done:
        return
    for obj in list(_closers):
        try:
            obj.close()
        except Exception:  # teardown goes on: every engine must still be destroyed
            pass
    # no thread of ours may still be inside a copy into a page-locked buffer or an engine call when the engines and
    # the buffers go: the PCM copy pool is joined, then every engine's streams and the device drained (VERDICT r5
    # next #2) before aid_engine_destroy (which also takes each engine's lock: a call still running finishes first)
    pool, _copy_pool = _copy_pool, None
    if pool is not None:
        try:
            pool.shutdown(wait=True)
        except Exception:
            pass
    for e in list(_live):
        try:
            e.sync()
        except Exception:
            pass
    try:
        import torch

        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
    except Exception:
        pass
    for e in list(_live):
        try:
            e.close()
        except Exception:
            pass
    for sl in list(_pinned_slots):
        sl.buf = None
    try:
        import torch

        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
            torch._C._host_emptyCache()  # page-locked blocks back to the runtime while it is alive
    except Exception:
        pass
    _shutdown_done = True


def _register_hook() -> None:
    global _hook_registered
    with _hook_lock:
        if _hook_registered:
            return
        try:  # torch registers its atexit handlers at import: import it first, so this hook runs before them
            import torch  # noqa: F401
        except ImportError:
            pass
        atexit.register(_shutdown)
        _hook_registered = True


_COPY_THREADS = int(os.environ.get("AIDFP_COPY_THREADS", 4))  # PCM copy threads; 8 lost 10-16 % at 64 clients (r06aj)
# floats (8 MiB): smaller batches are copied by the calling thread alone. Round 5 (profiles/r05w5_service_copy_ab.jsonl,
# whole 20 MB batches at 64 clients): threaded 26.6-27.5 k qps against 24.9-26.4 k single-threaded, and from 4 MiB the
# 16-client batches (5 MB) lost 7-10 %. Round 6 splits a 64-request batch into two 10 MB halves, which a 16 MiB bound
# left single-threaded: 8 MiB gives 33.1-34.0 k qps against 30.1-33.9 k (profiles/r06ai_service_copy_min_ab.jsonl).
# AIDFP_COPY_MIN_FLOATS overrides it (A/B runs)
_COPY_MIN = int(os.environ.get("AIDFP_COPY_MIN_FLOATS", 1 << 21))
_copy_pool = None
_copy_pool_lock = threading.Lock()


def _concat_into(arrs: list[np.ndarray], out: np.ndarray) -> None:
    """np.concatenate(arrs, out=out), split over a few threads for large batches: a coalesced batch of 64 five-second
    16 kHz queries is 20 MB, which one thread copies in ~2-4 ms -- most of a service batch's host time -- while
    numpy releases the GIL inside each slice assignment."""
    global _copy_pool
    if len(out) < _COPY_MIN or len(arrs) < 2 * _COPY_THREADS:
        np.concatenate(arrs, out=out)
        return
    if _copy_pool is None:
        with _copy_pool_lock:
            if _copy_pool is None:
                from concurrent.futures import ThreadPoolExecutor

                _copy_pool = ThreadPoolExecutor(_COPY_THREADS, thread_name_prefix="aidfp-pcm-copy")
    ends = np.cumsum([len(a) for a in arrs])

    def part(k: int) -> None:
        for i in range(k, len(arrs), _COPY_THREADS):
            out[ends[i] - len(arrs[i]): ends[i]] = arrs[i]

    for f in [_copy_pool.submit(part, k) for k in range(_COPY_THREADS)]:
        f.result()


def _new_slot() -> _PinnedSlot:
    sl = _PinnedSlot()
    _pinned_slots.add(sl)
    return sl


def _host_concat(arrs: list[np.ndarray], total: int, slot: "_PinnedSlot | None" = None) -> np.ndarray:
    """The clips concatenated into one host array for AID_PCM_HOST. Up to _PINNED_MAX samples it is a page-locked
    buffer (grown on demand), so the engine's single H2D copy of the span runs as a DMA instead of through the
    runtime's pageable staging (coalesced service queries). By default the calling thread's buffer: the engine call
    has finished with it when it returns (every synchronous host-PCM entry point syncs before returning its results);
    a submitted query passes its own `slot`, held until it is collected."""
    if total == 0:
        return np.zeros(1, dtype=np.float32)
    if total <= _PINNED_MAX:
        try:
            import torch

            sl = slot
            if sl is None:
                sl = getattr(_pinned, "slot", None)
                if sl is None:
                    sl = _pinned.slot = _new_slot()
            buf = sl.buf
            if buf is None or buf.numel() < total:
                if _finalizing():
                    raise RuntimeError("interpreter shutting down")
                buf = sl.buf = torch.empty(max(total, 1 << 20), dtype=torch.float32, pin_memory=True)
            out = buf.numpy()[:total]
            _concat_into(arrs, out)
            return out
        except (ImportError, RuntimeError):  # no torch / no device: pageable memory works the same, slower
            pass
    return np.concatenate(arrs)


class Engine:
    def __init__(self, sample_rate: int, hop: int = 0, peak_threshold: float = 0.0, device: int = -1,
                 min_match: int = 0, max_results: int = 0, keep_power: bool = False):
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
        if keep_power:  # parity/debug: the whole power plane for power() (K1 otherwise skips cold blocks)
            cfg.flags |= L.AID_FLAG_KEEP_POWER
        _register_hook()
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
        self._free_slots: list[_PinnedSlot] = []  # page-locked PCM buffers of collected submitted queries
        self._slot_lock = threading.Lock()
        _live.add(self)

    # -- lifecycle --
    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.aid_engine_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        if _finalizing():  # the ordered teardown (_shutdown) already destroyed every live engine
            return
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    FORCE = {"k5_path": L.AID_FORCE_K5_PATH, "k5_parts": L.AID_FORCE_K5_PARTS, "k5_batch": L.AID_FORCE_K5_BATCH,
             "k2_strips_x100": L.AID_FORCE_K2_STRIPS_X100, "k4_build": L.AID_FORCE_K4_BUILD,
             "exchange_fail": L.AID_FORCE_EXCHANGE_FAIL, "lane_gather": L.AID_FORCE_LANE_GATHER,
             "plane_rows": L.AID_FORCE_PLANE_ROWS}

    def force(self, what: str, value: int) -> None:
        """Test hook (aid_engine_force): pin one of the engine's own code paths, e.g. force("k5_path", 2)."""
        check(self._lib.aid_engine_force(self._h, self.FORCE[what], int(value)))

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
        pcm = _host_concat(arrs, int(offsets[-1]))
        check(self._lib.aid_extract(self._h, _p(pcm), _p(offsets), len(arrs), AID_PCM_HOST, None))
        self.n_clips = len(arrs)
        return [self.hashes(c) for c in range(len(arrs))]

    def extract_device(self, pcm_ptr: int, offsets: np.ndarray, stream: int | None = None) -> None:
        """Asynchronous extraction of device PCM; offsets = host int64[n_clips+1] (odd offsets allowed)."""
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
              stream: int | None = None, fmax_hz: int = 8000, sample_rate: int = 0, envelope: bool = True,
              wait: bool = True) -> None:
        """aidfp.synth's PCM into device memory [n_clips][n] (partials in [100, fmax_hz) Hz), sampled at
        `sample_rate` (0 = the engine's rate); envelope=False: the v0 stationary notes. wait=False returns once
        the generation is enqueued on `stream` (AID_SYNTH_ASYNC): the caller orders its reads on that stream."""
        tr = np.ascontiguousarray(tracks, dtype=np.uint32)
        st = np.ascontiguousarray(starts, dtype=np.int64)
        check(self._lib.aid_synth_rate(self._h, ctypes.c_void_p(dst_ptr), _p(tr), _p(st), len(tr), int(n),
                                       int(sample_rate) or self.sample_rate, int(noise_a), int(salt) & 0xFFFFFFFF,
                                       int(fmax_hz), (0 if envelope else L.AID_SYNTH_STATIONARY)
                                       | (0 if wait else L.AID_SYNTH_ASYNC),
                                       ctypes.c_void_p(stream) if stream else None))

    # -- index + match (FPSPEC 7) --
    def index_reset(self) -> None:
        check(self._lib.aid_index_reset(self._h))

    def index_add_extracted(self, track_ids) -> None:
        """Index every clip of the last extraction under track_ids[c]."""
        tr = np.ascontiguousarray(track_ids, dtype=np.uint32)
        if len(tr) != self.n_clips:
            raise ValueError("one track id per extracted clip")
        check(self._lib.aid_index_add_extracted(self._h, _p(tr)))

    def index_add_records(self, track: int, records: np.ndarray) -> None:
        """Index host records (uint64 hash | t1 << 32) as track `track`."""
        rec = np.ascontiguousarray(records, dtype=np.uint64)
        h = np.ascontiguousarray((rec & np.uint64(0xFFFFFFFF)).astype(np.uint32))
        t = np.ascontiguousarray((rec >> np.uint64(32)).astype(np.uint32))
        tr = np.full(len(rec), track, dtype=np.uint32)
        if len(rec) == 0:  # no hashes (short/quiet clip): the id still gets a slot, so it can be removed
            check(self._lib.aid_index_add_track(self._h, int(track)))
            return
        check(self._lib.aid_index_add_postings(self._h, _p(h), _p(tr), _p(t), len(rec), AID_PCM_HOST))

    def index_add_postings(self, hash_ptr: int, track_ptr: int, t_ptr: int, n: int, device: bool = True) -> None:
        check(self._lib.aid_index_add_postings(self._h, ctypes.c_void_p(hash_ptr), ctypes.c_void_p(track_ptr),
                                               ctypes.c_void_p(t_ptr), int(n), AID_PCM_DEVICE if device else AID_PCM_HOST))

    def index_remove(self, track: int) -> None:
        check(self._lib.aid_index_remove(self._h, int(track)))

    def index_compact(self) -> int:
        """Drop the stored postings of removed tracks; returns how many were dropped."""
        n = ctypes.c_int64()
        check(self._lib.aid_index_compact(self._h, ctypes.byref(n)))
        return int(n.value)

    def index_finalize(self) -> None:
        check(self._lib.aid_index_finalize(self._h))

    def index_stats(self) -> dict:
        n = ctypes.c_int64()
        live = ctypes.c_int64()
        nt = ctypes.c_uint32()
        check(self._lib.aid_index_stats(self._h, ctypes.byref(n), ctypes.byref(live), ctypes.byref(nt)))
        return {"postings": n.value, "live": live.value, "tracks": nt.value}

    def match_stats(self, reset: bool = False) -> dict:
        """Cumulative K5 counters (aid_match_stats): queries, votes, postings read, path split, records."""
        out = np.zeros(13, dtype=np.int64)
        check(self._lib.aid_match_stats(self._h, _p(out), 13, 1 if reset else 0))
        return dict(zip(("queries", "votes", "posting_reads", "queries_lds", "queries_global", "records", "sig_reads",
                         "lds_path_workgroups_per_cu", "fallback_heavy", "fallback_table", "fallback_distinct",
                         "fallback_tracks", "fallback_rows"), (int(x) for x in out)))

    # ---- PCM front-end (FPSPEC 8): downmix + resample, device buffers ----
    def resample_len(self, n: int, sr_in: int, sr_out: int) -> int:
        return int(self._lib.aid_resample_len(int(n), int(sr_in), int(sr_out)))

    def resample(self, src_ptr: int, n: int, channels: int, sr_in: int, sr_out: int, dst_ptr: int, cap: int,
                 stream: int | None = None) -> int:
        """Asynchronous: n frames of `channels` floats at sr_in -> mono at sr_out; returns the output length."""
        m = ctypes.c_int64(0)
        check(self._lib.aid_resample(self._h, ctypes.c_void_p(src_ptr), int(n), int(channels), int(sr_in),
                                     int(sr_out), ctypes.c_void_p(dst_ptr), int(cap), ctypes.byref(m),
                                     ctypes.c_void_p(stream) if stream else None))
        return int(m.value)

    def resample_range(self, src_ptr: int, in_base: int, n: int, channels: int, sr_in: int, sr_out: int,
                       m_first: int, count: int, dst_ptr: int, stream: int | None = None) -> None:
        """Streaming form: stream outputs [m_first, m_first+count) from src (= stream samples
        [in_base, in_base+n)); see include/aidfp.h."""
        check(self._lib.aid_resample_range(self._h, ctypes.c_void_p(src_ptr), int(in_base), int(n), int(channels),
                                           int(sr_in), int(sr_out), int(m_first), int(count),
                                           ctypes.c_void_p(dst_ptr), ctypes.c_void_p(stream) if stream else None))

    def resample_batch(self, src_ptr: int, src_stride: int, n_streams: int, in_base: int, n: int, channels: int,
                       sr_in: int, sr_out: int, m_first: int, count: int, dst_ptr: int, dst_stride: int,
                       stream: int | None = None) -> None:
        """resample_range for n_streams lockstep streams in one launch (strides in floats; aid_resample_batch)."""
        check(self._lib.aid_resample_batch(self._h, ctypes.c_void_p(src_ptr), int(src_stride), int(n_streams),
                                           int(in_base), int(n), int(channels), int(sr_in), int(sr_out), int(m_first),
                                           int(count), ctypes.c_void_p(dst_ptr), int(dst_stride),
                                           ctypes.c_void_p(stream) if stream else None))

    def resample_batch_split(self, hist_ptr: int, hist_stride: int, hist_n: int, src_ptr: int, src_stride: int,
                             n_streams: int, in_base: int, n: int, channels: int, sr_in: int, sr_out: int, m_first: int,
                             count: int, dst_ptr: int, dst_stride: int, stream: int | None = None) -> None:
        """resample_batch over stream frames [in_base - hist_n, in_base) at hist_ptr then [in_base, in_base + n) at
        src_ptr (aid_resample_batch_split): a chunk is read in place, only its predecessor's tail is kept."""
        check(self._lib.aid_resample_batch_split(self._h, ctypes.c_void_p(hist_ptr), int(hist_stride), int(hist_n),
                                                 ctypes.c_void_p(src_ptr), int(src_stride), int(n_streams),
                                                 int(in_base), int(n), int(channels), int(sr_in), int(sr_out),
                                                 int(m_first), int(count), ctypes.c_void_p(dst_ptr), int(dst_stride),
                                                 ctypes.c_void_p(stream) if stream else None))

    def resample_plan(self, sr_in: int, sr_out: int):
        v = [ctypes.c_int32() for _ in range(4)]
        if not self._lib.aid_resample_plan(int(sr_in), int(sr_out), *[ctypes.byref(x) for x in v]):
            raise ValueError("bad sample rates")
        return tuple(x.value for x in v)  # up, down, hl, J

    # ---- native RCCL exchange (aid_comm_*, aid_index_allgather) ----
    def comm_id(self) -> bytes:
        """RCCL unique id (128 bytes) for aid_comm_create; made by rank 0, shared by the host."""
        buf = (ctypes.c_uint8 * 128)()
        check(self._lib.aid_comm_id(buf))
        return bytes(buf)

    def comm_create(self, comm_id: bytes, world: int, rank: int) -> int:
        if len(comm_id) != 128:
            raise ValueError("comm id must be 128 bytes")
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(comm_id)
        check(self._lib.aid_comm_create(self._h, buf, int(world), int(rank), ctypes.byref(h)))
        return h.value

    def comm_destroy(self, comm: int) -> None:
        if comm:
            self._lib.aid_comm_destroy(ctypes.c_void_p(comm))

    def index_allgather(self, comm: int, first: int = 0) -> int:
        """Collective: replace postings [first, n) by the union of every rank's [first, n)."""
        n = ctypes.c_int64(0)
        check(self._lib.aid_index_allgather(self._h, ctypes.c_void_p(comm), int(first), ctypes.byref(n)))
        return int(n.value)

    def comm_size(self, comm: int) -> tuple[int, int]:
        """(ranks, this rank) as the RCCL communicator sees them (ncclCommCount / ncclCommUserRank)."""
        w, r = ctypes.c_int32(), ctypes.c_int32()
        check(self._lib.aid_comm_size(ctypes.c_void_p(comm), ctypes.byref(w), ctypes.byref(r)))
        return int(w.value), int(r.value)

    def index_shard_info(self, first: int = 0) -> tuple[int, int]:
        """(postings in [first, n), n_tracks): what this rank contributes to an index exchange."""
        n, nt = ctypes.c_int64(), ctypes.c_uint32()
        check(self._lib.aid_index_shard_info(self._h, int(first), ctypes.byref(n), ctypes.byref(nt)))
        return int(n.value), int(nt.value)

    def index_reserve(self, first: int, total: int, n_tracks: int, stream: int | None = None) -> None:
        """Grow the posting planes / track tables for a splice of `total` postings at `first` (index unchanged)."""
        check(self._lib.aid_index_reserve(self._h, int(first), int(total), int(n_tracks),
                                          ctypes.c_void_p(stream) if stream else None))

    def index_pack(self, first: int, planes_ptr: int, stride: int, stream: int | None = None) -> None:
        """Copy this rank's shard [first, n) into device planes [3][stride] (hash, track, t; zero padded)."""
        check(self._lib.aid_index_pack(self._h, int(first), ctypes.c_void_p(planes_ptr), int(stride),
                                       ctypes.c_void_p(stream) if stream else None))

    def index_splice(self, first: int, recv_ptr: int, counts, stride: int, n_tracks: int,
                     stream: int | None = None) -> int:
        """Replace [first, n) by the gathered shards (device recv [world][3][stride]); failure-atomic."""
        c = np.ascontiguousarray(counts, dtype=np.int64)
        check(self._lib.aid_index_splice(self._h, int(first), ctypes.c_void_p(recv_ptr), len(c), int(stride), _p(c),
                                         int(n_tracks), ctypes.c_void_p(stream) if stream else None))
        return self.index_stats()["postings"]

    def index_export(self, first: int = 0, count: int | None = None) -> np.ndarray:
        """Host copy of stored postings [first, first+count) as [n, 3] uint32 (hash, track, t)."""
        total = self.index_stats()["postings"]
        count = total - first if count is None else count
        cols = [np.zeros(max(count, 1), dtype=np.uint32) for _ in range(3)]
        check(self._lib.aid_index_export(self._h, _p(cols[0]), _p(cols[1]), _p(cols[2]), first, count, AID_PCM_HOST))
        return np.stack([c[:count] for c in cols], axis=1)

    def index_checksum(self, first: int = 0, count: int | None = None) -> int:
        """aid_index_checksum: order-sensitive 64-bit checksum of stored postings [first, first+count) (device)."""
        count = self.index_stats()["postings"] - first if count is None else count
        out = ctypes.c_uint64(0)
        check(self._lib.aid_index_checksum(self._h, int(first), int(count), ctypes.byref(out)))
        return int(out.value)

    def index_csr(self, offsets: bool = True) -> tuple[np.ndarray | None, np.ndarray]:
        """aid_index_csr_export: the finalized CSR as (offsets u32 [2^26 + 1] or None, posts u64 [n])."""
        n = ctypes.c_int64(0)
        check(self._lib.aid_index_csr_export(self._h, None, 0, None, 0, ctypes.byref(n)))
        posts = np.empty(int(n.value), np.uint64)
        offs = np.empty((1 << 26) + 1, np.uint32) if offsets else None
        check(self._lib.aid_index_csr_export(self._h, None if offs is None else offs.ctypes.data_as(ctypes.c_void_p),
                                             0 if offs is None else len(offs),
                                             posts.ctypes.data_as(ctypes.c_void_p), len(posts), ctypes.byref(n)))
        return offs, posts

    def index_export_device(self, hash_ptr: int, track_ptr: int, t_ptr: int, first: int, count: int) -> None:
        check(self._lib.aid_index_export(self._h, ctypes.c_void_p(hash_ptr), ctypes.c_void_p(track_ptr),
                                         ctypes.c_void_p(t_ptr), first, count, AID_PCM_DEVICE))

    def index_save(self, path: str) -> None:
        check(self._lib.aid_index_save(self._h, str(path).encode()))

    def index_load(self, path: str) -> None:
        check(self._lib.aid_index_load(self._h, str(path).encode()))

    def _row_buf(self, nq: int) -> np.ndarray:
        """Host rows [nq][max_results] of aid_match_row (5 int32 each) as a plain int32 array: np.ctypeslib.as_array
        of a ctypes Structure array parsed its PEP 3118 format on every call (~40 us per query call)."""
        return np.empty(max(1, nq * self.max_results) * 5, dtype=np.int32)

    def _rows(self, rows: np.ndarray, nrows, nq: int) -> list[np.ndarray]:
        # one conversion for the batch, then per-query views (a per-query astype cost ~1 us each)
        arr = rows[: nq * self.max_results * 5].reshape(nq, self.max_results, 5).astype(np.int64)
        return [r[:k] for r, k in zip(arr, nrows.tolist())]

    def query(self, queries) -> list[np.ndarray]:
        """Match host record arrays; per query [r, 5] int64 rows (count, track, d, tq_min, tq_max)."""
        qs = [np.ascontiguousarray(q, dtype=np.uint64).ravel() for q in queries]
        nq = len(qs)
        if nq == 0:
            return []
        qoff = np.zeros(nq + 1, dtype=np.int64)
        qoff[1:] = np.cumsum([len(q) for q in qs])
        recs = np.concatenate(qs) if qoff[-1] else np.zeros(1, dtype=np.uint64)
        rows = self._row_buf(nq)
        nrows = np.zeros(nq, dtype=np.int32)
        check(self._lib.aid_query(self._h, _p(recs), _p(qoff), nq, rows.ctypes.data, _p(nrows)))
        return self._rows(rows, nrows, nq)

    def query_extracted(self) -> list[np.ndarray]:
        """Match every clip of the last extraction (records never leave the device)."""
        nq = self.n_clips
        if nq == 0:
            return []
        rows = self._row_buf(nq)
        nrows = np.zeros(nq, dtype=np.int32)
        check(self._lib.aid_query_extracted(self._h, rows.ctypes.data, _p(nrows)))
        return self._rows(rows, nrows, nq)

    def query_pcm(self, clips: Sequence[np.ndarray]) -> list[np.ndarray]:
        """Extract + match host clips in one engine call (aid_query_pcm; thread-safe as a unit)."""
        arrs = [np.ascontiguousarray(c, dtype=np.float32).ravel() for c in clips]
        nq = len(arrs)
        if nq == 0:
            return []
        offsets = np.zeros(nq + 1, dtype=np.int64)
        offsets[1:] = np.cumsum([len(a) for a in arrs])
        pcm = _host_concat(arrs, int(offsets[-1]))
        rows = self._row_buf(nq)
        nrows = np.zeros(nq, dtype=np.int32)
        check(self._lib.aid_query_pcm(self._h, _p(pcm), _p(offsets), nq, AID_PCM_HOST, rows.ctypes.data,
                                      _p(nrows), None))
        self.n_clips = nq
        return self._rows(rows, nrows, nq)

    def query_pcm_submit(self, clips: Sequence[np.ndarray]) -> "PendingQuery":
        """query_pcm in two halves (aid_query_pcm_submit): the batch is laid into a page-locked buffer of its own,
        its copy, extraction, K5 and result copies are queued, and a PendingQuery is returned at once; collect()
        waits and returns the rows (the buffer is reused after that). A caller submits batch N + 1 before it
        collects batch N (QueryCoalescer's pipelined dispatch)."""
        arrs = [np.ascontiguousarray(c, dtype=np.float32).ravel() for c in clips]
        nq = len(arrs)
        offsets = np.zeros(nq + 1, dtype=np.int64)
        if nq:
            offsets[1:] = np.cumsum([len(a) for a in arrs])
        with self._slot_lock:
            slot = self._free_slots.pop() if self._free_slots else _new_slot()
        try:
            pcm = _host_concat(arrs, int(offsets[-1]), slot)
            t = ctypes.c_void_p()
            check(self._lib.aid_query_pcm_submit(self._h, _p(pcm), _p(offsets), nq, AID_PCM_HOST, None,
                                                 ctypes.byref(t)))
        except BaseException:
            self._put_slot(slot)  # a failed submit has drained its copy (drain_host_copy)
            raise
        return PendingQuery(self, t, nq, slot, pcm)

    def _put_slot(self, slot) -> None:
        with self._slot_lock:
            if len(self._free_slots) < 4:
                self._free_slots.append(slot)

    def query_windows(self, pcm_ptr: int, starts, ends, stream: int | None = None) -> list[np.ndarray]:
        """Extract + match device-PCM windows [starts[c], ends[c]) (may overlap) in one engine call."""
        st = np.ascontiguousarray(starts, dtype=np.int64)
        en = np.ascontiguousarray(ends, dtype=np.int64)
        nq = len(st)
        if nq == 0:
            return []
        rows = self._row_buf(nq)
        nrows = np.zeros(nq, dtype=np.int32)
        check(self._lib.aid_query_windows(self._h, ctypes.c_void_p(pcm_ptr), _p(st), _p(en), nq, rows.ctypes.data,
                                          _p(nrows), ctypes.c_void_p(stream) if stream else None))
        self.n_clips = nq
        return self._rows(rows, nrows, nq)

    def query_windows_submit(self, pcm_ptr: int, starts, ends, stream: int | None = None) -> "PendingQuery":
        """query_windows in two halves (aid_query_windows_submit): the extraction, K5 and the result copies are queued
        on `stream` and a PendingQuery is returned at once; its collect() waits for them and returns the rows."""
        st = np.ascontiguousarray(starts, dtype=np.int64)
        en = np.ascontiguousarray(ends, dtype=np.int64)
        t = ctypes.c_void_p()
        check(self._lib.aid_query_windows_submit(self._h, ctypes.c_void_p(pcm_ptr), _p(st), _p(en), len(st),
                                                 ctypes.c_void_p(stream) if stream else None, ctypes.byref(t)))
        return PendingQuery(self, t, len(st))

    # -- batched exact lane --
    EXACT_DTYPE = np.dtype([("track", "<u4"), ("aligned_hashes", "<i4"), ("offset_seconds", "<f8"),
                            ("confidence", "<f8")])

    def exact_lane(self, clips: Sequence[np.ndarray] | None = None, max_out: int = 0, *, pcm_ptr: int = 0,
                   offsets: np.ndarray | None = None) -> list[np.ndarray]:
        """Sub-window fan-out + match + consensus + ranking for a batch of clips (aid_exact_lane).

        Host clips, or device PCM (pcm_ptr) with host offsets. Returns per clip a structured array
        (track, aligned_hashes, offset_seconds, confidence) in rank order, at most max_out rows
        (default 3 x max_results: every candidate the consensus can keep)."""
        max_out = int(max_out) or 3 * self.max_results
        if clips is not None:
            arrs = [np.ascontiguousarray(c, dtype=np.float32).ravel() for c in clips]
            offsets = np.zeros(len(arrs) + 1, dtype=np.int64)
            if arrs:
                offsets[1:] = np.cumsum([len(a) for a in arrs])
            pcm = _host_concat(arrs, int(offsets[-1]))
            src, loc = _p(pcm), AID_PCM_HOST
        else:
            offsets = np.ascontiguousarray(offsets, dtype=np.int64)
            src, loc = ctypes.c_void_p(pcm_ptr), AID_PCM_DEVICE
        n = len(offsets) - 1
        if n <= 0:
            return []
        out = np.zeros(n * max_out, dtype=self.EXACT_DTYPE)
        nout = np.zeros(n, dtype=np.int32)
        check(self._lib.aid_exact_lane(self._h, src, _p(offsets), n, loc, max_out, _p(out), _p(nout), None))
        # per-clip views of the one result array (4096 per-clip copies took ~3.5 ms of host time per lane call)
        return [r[:k] for r, k in zip(out.reshape(n, max_out), nout.tolist())]

    def downmix(self, stereo_ptr: int, n_frames: int, mono_ptr: int, stream: int | None = None) -> None:
        check(self._lib.aid_downmix(self._h, ctypes.c_void_p(stereo_ptr), int(n_frames), ctypes.c_void_p(mono_ptr),
                                    ctypes.c_void_p(stream) if stream else None))

    # -- profiling --
    def profile_enable(self, on: bool = True) -> None:
        check(self._lib.aid_profile_enable(self._h, 1 if on else 0))

    def profile_select(self, kernels) -> None:
        """Restrict profiling events to these kernel ids (AID_K_*); None = all."""
        mask = 0xFFFFFFFF if kernels is None else sum(1 << int(k) for k in kernels)
        check(self._lib.aid_profile_select(self._h, ctypes.c_uint32(mask)))

    def profile_read(self, reset: bool = False) -> dict:
        ms = np.zeros(L.AID_K_COUNT, dtype=np.float64)
        n = np.zeros(L.AID_K_COUNT, dtype=np.int64)
        check(self._lib.aid_profile_read(self._h, _p(ms), _p(n), 1 if reset else 0))
        return {name: (float(ms[i]), int(n[i])) for i, name in enumerate(L.KERNEL_NAMES)}


def exact_windows(n: int, sample_rate: int) -> tuple[int, list[tuple[int, int]]]:
    """The exact lane's window plan for a clip of n samples (host only): (mode, [(lo, len)])."""
    lo = np.zeros(3, dtype=np.int64)
    ln = np.zeros(3, dtype=np.int64)
    mode = np.zeros(1, dtype=np.int32)
    k = L.load().aid_exact_windows(int(n), int(sample_rate), _p(lo), _p(ln), _p(mode))
    if k < 0:
        raise EngineError(k, L.last_error())
    return int(mode[0]), [(int(lo[w]), int(ln[w])) for w in range(k)]


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


class PendingQuery:
    """A submitted aid_query_windows_submit / aid_query_pcm_submit ticket; collect() once (a dropped one is collected
    and discarded). A host-PCM ticket holds its page-locked buffer (and the array over it) until collected."""

    __slots__ = ("eng", "ticket", "nq", "slot", "pcm")

    def __init__(self, eng: "Engine", ticket: ctypes.c_void_p, nq: int, slot=None, pcm=None):
        self.eng, self.ticket, self.nq, self.slot, self.pcm = eng, ticket, nq, slot, pcm

    def collect(self) -> list[np.ndarray]:
        if self.ticket is None:
            raise RuntimeError("ticket already collected")
        t, self.ticket = self.ticket, None
        nq = self.nq
        mr = self.eng.max_results
        rows = self.eng._row_buf(nq)
        nrows = np.zeros(max(1, nq), dtype=np.int32)
        try:
            check(self.eng._lib.aid_query_windows_collect(self.eng._h, t, rows.ctypes.data, _p(nrows)))
        finally:  # collect waited for the ticket's work (also on error): its PCM buffer is free again
            slot, self.slot, self.pcm = self.slot, None, None
            if slot is not None:
                self.eng._put_slot(slot)
        return self.eng._rows(rows, nrows[:nq], nq) if nq else []

    def __del__(self):  # pragma: no cover - an abandoned ticket still frees its buffers
        if getattr(self, "ticket", None) is not None and not _finalizing():
            try:
                self.collect()
            except Exception:
                pass
