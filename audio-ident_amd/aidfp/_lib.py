"""ctypes binding of libaidfp.so (include/aidfp.h).

The library is the product path: if it is missing or fails to load, every
engine call raises ``EngineUnavailable`` -- there is no CPU fallback.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_PATH = Path(os.environ.get("AIDFP_LIB", Path(__file__).resolve().parent / "libaidfp.so"))

AID_OK = 0
AID_ERR_INVALID = -1
AID_ERR_DEVICE = -2
AID_ERR_NOMEM = -3
AID_ERR_STATE = -4
AID_PCM_HOST = 0
AID_PCM_DEVICE = 1
AID_FLAG_KEEP_POWER = 1
AID_SYNTH_STATIONARY = 1
AID_SYNTH_ASYNC = 2
(AID_FORCE_K5_PATH, AID_FORCE_K5_PARTS, AID_FORCE_K5_BATCH, AID_FORCE_K2_STRIPS_X100, AID_FORCE_K4_BUILD,
 AID_FORCE_EXCHANGE_FAIL, AID_FORCE_LANE_GATHER, AID_FORCE_PLANE_ROWS) = 1, 2, 3, 4, 5, 6, 7, 8
AID_K_STFT, AID_K_PEAKS, AID_K_LANDMARK_COUNT, AID_K_LANDMARK_WRITE, AID_K_SYNTH, AID_K_MATCH = range(6)
AID_K_COUNT = 12
KERNEL_NAMES = ["stft_power", "peak_pick", "landmark_count", "landmark_write", "synth", "match", "resample",
                "dedup", "index_build", "vote_hist", "hot_scan", "vote_final"]


class EngineUnavailable(RuntimeError):
    """libaidfp.so could not be loaded or the GPU could not be initialised."""


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"aidfp error {code}: {msg}")
        self.code = code


class AidConfig(ctypes.Structure):
    _fields_ = [
        ("sample_rate", ctypes.c_int32),
        ("hop", ctypes.c_int32),
        ("peak_threshold", ctypes.c_float),
        ("device", ctypes.c_int32),
        ("min_match", ctypes.c_int32),
        ("max_results", ctypes.c_int32),
        ("flags", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 9),
    ]


class AidHash(ctypes.Structure):
    _fields_ = [("hash", ctypes.c_uint32), ("t1", ctypes.c_uint32)]


class AidMatchRow(ctypes.Structure):
    _fields_ = [
        ("match_count", ctypes.c_int32),
        ("track", ctypes.c_uint32),
        ("d", ctypes.c_int32),
        ("tq_min", ctypes.c_int32),
        ("tq_max", ctypes.c_int32),
    ]


class AidExactRow(ctypes.Structure):
    _fields_ = [
        ("track", ctypes.c_uint32),
        ("aligned_hashes", ctypes.c_int32),
        ("offset_seconds", ctypes.c_double),
        ("confidence", ctypes.c_double),
    ]


# (name, restype, argtypes) for every symbol include/aidfp.h declares
P = ctypes.c_void_p
I32 = ctypes.c_int32
I64 = ctypes.c_int64
SIGNATURES = [
    ("aid_abi_version", I32, []),
    ("aid_last_error", ctypes.c_char_p, []),
    ("aid_config_default", ctypes.c_int, [I32, P]),
    ("aid_engine_create", ctypes.c_int, [P, P]),
    ("aid_engine_destroy", None, [P]),
    ("aid_engine_config", ctypes.c_int, [P, P]),
    ("aid_engine_force", ctypes.c_int, [P, I32, I32]),
    ("aid_num_frames", I64, [P, I64]),
    ("aid_hash_capacity", I64, [P, I64]),
    ("aid_extract", ctypes.c_int, [P, P, P, I32, I32, P]),
    ("aid_sync", ctypes.c_int, [P]),
    ("aid_result_counts", ctypes.c_int, [P, P]),
    ("aid_result_hashes", ctypes.c_int, [P, I32, P, I64, P]),
    ("aid_result_device", ctypes.c_int, [P, P, P, P, P]),
    ("aid_result_power", ctypes.c_int, [P, I32, P, I64]),
    ("aid_result_peakmask", ctypes.c_int, [P, I32, P, I64]),
    ("aid_spectrogram", ctypes.c_int, [P, P, I64, P, I64]),
    ("aid_synth", ctypes.c_int, [P, P, P, P, I32, I64, I32, ctypes.c_uint32, P]),
    ("aid_synth_band", ctypes.c_int, [P, P, P, P, I32, I64, I32, ctypes.c_uint32, I32, P]),
    ("aid_synth_rate", ctypes.c_int, [P, P, P, P, I32, I64, I32, I32, ctypes.c_uint32, I32, I32, P]),
    ("aid_index_reset", ctypes.c_int, [P]),
    ("aid_index_add_extracted", ctypes.c_int, [P, P]),
    ("aid_index_add_postings", ctypes.c_int, [P, P, P, P, I64, I32]),
    ("aid_index_add_track", ctypes.c_int, [P, ctypes.c_uint32]),
    ("aid_index_remove", ctypes.c_int, [P, ctypes.c_uint32]),
    ("aid_index_compact", ctypes.c_int, [P, P]),
    ("aid_index_finalize", ctypes.c_int, [P]),
    ("aid_index_stats", ctypes.c_int, [P, P, P, P]),
    ("aid_match_stats", ctypes.c_int, [P, P, I32, I32]),
    ("aid_index_export", ctypes.c_int, [P, P, P, P, I64, I64, I32]),
    ("aid_index_checksum", ctypes.c_int, [P, I64, I64, P]),
    ("aid_index_csr_export", ctypes.c_int, [P, P, I64, P, I64, P]),
    ("aid_comm_id", ctypes.c_int, [P]),
    ("aid_comm_create", ctypes.c_int, [P, P, I32, I32, P]),
    ("aid_comm_destroy", None, [P]),
    ("aid_index_allgather", ctypes.c_int, [P, P, I64, P]),
    ("aid_comm_size", ctypes.c_int, [P, P, P]),
    ("aid_index_shard_info", ctypes.c_int, [P, I64, P, P]),
    ("aid_index_reserve", ctypes.c_int, [P, I64, I64, ctypes.c_uint32, P]),
    ("aid_index_pack", ctypes.c_int, [P, I64, P, I64, P]),
    ("aid_index_splice", ctypes.c_int, [P, I64, P, I32, I64, P, ctypes.c_uint32, P]),
    ("aid_index_save", ctypes.c_int, [P, ctypes.c_char_p]),
    ("aid_index_load", ctypes.c_int, [P, ctypes.c_char_p]),
    ("aid_query", ctypes.c_int, [P, P, P, I32, P, P]),
    ("aid_query_extracted", ctypes.c_int, [P, P, P]),
    ("aid_query_pcm", ctypes.c_int, [P, P, P, I32, I32, P, P, P]),
    ("aid_query_windows", ctypes.c_int, [P, P, P, P, I32, P, P, P]),
    ("aid_query_windows_submit", ctypes.c_int, [P, P, P, P, I32, P, P]),
    ("aid_query_windows_collect", ctypes.c_int, [P, P, P, P]),
    ("aid_query_pcm_submit", ctypes.c_int, [P, P, P, I32, I32, P, P]),
    ("aid_exact_lane", ctypes.c_int, [P, P, P, I32, I32, I32, P, P, P]),
    ("aid_exact_windows", ctypes.c_int, [I64, I32, P, P, P]),
    ("aid_downmix", ctypes.c_int, [P, P, I64, P, P]),
    ("aid_resample_len", I64, [I64, I32, I32]),
    ("aid_resample", ctypes.c_int, [P, P, I64, I32, I32, I32, P, I64, P, P]),
    ("aid_resample_range", ctypes.c_int, [P, P, I64, I64, I32, I32, I32, I64, I64, P, P]),
    ("aid_resample_batch", ctypes.c_int, [P, P, I64, I32, I64, I64, I32, I32, I32, I64, I64, P, I64, P]),
    ("aid_resample_batch_split", ctypes.c_int, [P, P, I64, I64, P, I64, I32, I64, I64, I32, I32, I32, I64, I64, P, I64, P]),
    ("aid_resample_plan", ctypes.c_int, [I32, I32, P, P, P, P]),
    ("aid_dedup_reset", ctypes.c_int, [P]),
    ("aid_dedup_add", ctypes.c_int, [P, P, P, P, I32]),
    ("aid_dedup_count", ctypes.c_int, [P, P, P]),
    ("aid_dedup_scan", ctypes.c_int, [P, P, P, P, I32, P, P]),
    ("aid_dedup_pairs", ctypes.c_int, [P, P, P, P, P, I32, P]),
    ("aid_profile_enable", ctypes.c_int, [P, I32]),
    ("aid_profile_read", ctypes.c_int, [P, P, P, I32]),
    ("aid_profile_select", ctypes.c_int, [P, ctypes.c_uint32]),
]

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise EngineUnavailable(f"{LIB_PATH} not built (run __graft_entry__.build())")
        # One HIP runtime per process: torch bundles its own libamdhip64.so.7. Loading torch
        # first makes the dynamic loader bind libaidfp's NEEDED libamdhip64.so.7 to that same
        # copy (SONAME match); loading ours first would put two runtimes in the process.
        try:
            import torch  # noqa: F401  (plumbing: device memory, streams, RCCL)
        except ImportError:  # pragma: no cover - torch is part of the image
            pass
        try:
            L = ctypes.CDLL(str(LIB_PATH))
        except OSError as exc:  # pragma: no cover - depends on the box
            raise EngineUnavailable(f"cannot load {LIB_PATH}: {exc}") from exc
        ab = "AIDFP_LIB" in os.environ  # an A/B build of an older source tree may lack newer entry points
        for name, res, args in SIGNATURES:
            try:
                f = getattr(L, name)
            except AttributeError:
                if ab:
                    continue
                raise
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    msg = load().aid_last_error()
    return msg.decode(errors="replace") if msg else ""


def check(rc: int) -> None:
    if rc != AID_OK:
        raise EngineError(rc, last_error())
