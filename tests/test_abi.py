"""The C-ABI library loads and exports every symbol include/aidfp.h declares (no GPU
calls), and the ctypes signature table covers exactly that set."""

import ctypes
import re
from pathlib import Path

from aidfp import _lib

HEADER = Path(__file__).resolve().parents[1] / "include" / "aidfp.h"


def declared():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(aid_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    names = declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_signature_table_matches_header():
    assert sorted(n for n, _, _ in _lib.SIGNATURES) == declared()


def test_abi_version_and_defaults_without_gpu():
    L = _lib.load()
    assert L.aid_abi_version() == 1
    cfg = _lib.AidConfig()
    assert L.aid_config_default(44100, ctypes.byref(cfg)) == 0
    assert (cfg.hop, cfg.min_match, cfg.max_results) == (512, 10, 50)  # FPSPEC v1 7
    assert abs(cfg.peak_threshold - 4.0) < 1e-9
    assert L.aid_config_default(16000, ctypes.byref(cfg)) == 0 and cfg.hop == 256
    assert L.aid_config_default(0, ctypes.byref(cfg)) == _lib.AID_ERR_INVALID
    assert "bad argument" in _lib.last_error()


def test_python_constants_match_header():
    """Every #define AID_* the Python side mirrors has the header's value (a stale
    AID_K_COUNT would make aid_profile_read write past the ctypes arrays)."""
    defs = dict(re.findall(r"#define\s+(AID_[A-Z0-9_]+)\s+(-?\d+)", HEADER.read_text()))
    mirrored = {k: getattr(_lib, k) for k in defs if hasattr(_lib, k)}
    assert "AID_K_COUNT" in mirrored and len(mirrored) >= 5
    for k, v in mirrored.items():
        assert v == int(defs[k]), k
    assert len(_lib.KERNEL_NAMES) == int(defs["AID_K_COUNT"])


def test_resample_len_without_gpu():
    L = _lib.load()
    assert L.aid_resample_len(48000, 48000, 16000) == 16000
    assert L.aid_resample_len(48001, 48000, 16000) == 16001
    assert L.aid_resample_len(1000, 44100, 48000) == 1089  # ceil(1000 * 160 / 147)
    assert L.aid_resample_len(0, 48000, 16000) == 0
    assert L.aid_resample_len(10, 0, 16000) == 0


def test_product_library_links_no_rocprim():
    """rocPRIM's radix sort is the K4 A/B reference of the diagnostic variant build only; the product
    library defines no symbol of it (its code would appear as rocprim:: template instances)."""
    import shutil
    import subprocess

    import pytest

    if not shutil.which("nm"):
        pytest.skip("nm not available")
    out = subprocess.run(["nm", "-C", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    assert "rocprim::" not in out
