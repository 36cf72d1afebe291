"""Build libaidfp.so (HIP, gfx950) in-tree: audio-ident_amd/aidfp/libaidfp.so.

One hipcc invocation per translation unit (parallel), then one link. Flags:
``-ffp-contract=off`` is load-bearing: spec/FPSPEC.md pins every binary32 op,
so hipcc must not fuse a multiply and an add on its own.
"""

from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "aidfp" / "libaidfp.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"

SOURCES = ["stft.hip", "peaks.hip", "landmarks.hip", "synth.hip", "index.hip", "index_sort.hip", "stream.hip",
           "resample.hip", "dedup.hip", "exact.hip", "engine.cpp"]
FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-ffp-contract=off",
    "-fno-fast-math",
    "-Wall",
    "-Wno-unused-result",
]
# Per-file flags. K1 is complex arithmetic whose DFT4 mixes re/im across lanes of a float2: hipcc's
# SLP vectorizer packs it into v_pk_*_f32 (4 cycles each on gfx950, the rate of two scalar ops) plus
# ~134 v_mov per frame to shuffle pairs; scalar code is 20 % fewer VALU cycles (K1 0.464 -> 0.419 ms,
# same-box A/B). K2 is the opposite (0.290 -> 0.329 without SLP), so this stays per file.
FILE_FLAGS = {"stft.hip": ["-fno-slp-vectorize"]}


def _deps(src: Path) -> list[Path]:
    return [src, Path(__file__)] + sorted(CSRC.glob("*.h")) + [PKG.parent / "include" / "aidfp.h"]


def _compile(name: str, verbose: bool, objdir: Path = OBJ, extra: tuple = ()) -> Path:
    src = CSRC / name
    obj = objdir / (name + ".o")
    if obj.exists() and all(d.stat().st_mtime <= obj.stat().st_mtime for d in _deps(src)):
        return obj
    flags = [*FLAGS, *FILE_FLAGS.get(name, []), *extra]
    cmd = [HIPCC, *flags, "-c", str(src), "-o", str(obj)]
    if name.endswith(".cpp"):
        cmd = [HIPCC, *flags, "-x", "hip", "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(verbose: bool = False, variant: str | None = None, defines: tuple = (), flags: tuple = ()) -> Path:
    """Build the product library; `variant` builds a diagnostic copy (build/<variant>/libaidfp.so)
    with extra -D defines, used only for profiling experiments (never loaded by default)."""
    objdir = OBJ if variant is None else OBJ / variant
    lib = LIB if variant is None else objdir / "libaidfp.so"
    objdir.mkdir(parents=True, exist_ok=True)
    extra = tuple(f"-D{d}" for d in defines) + tuple(flags)
    srcs = [s for s in SOURCES if (CSRC / s).exists()]
    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose, objdir, extra), srcs))
    if lib.exists() and all(o.stat().st_mtime <= lib.stat().st_mtime for o in objs):
        return lib
    # librccl.so.1: the same SONAME torch bundles, so one RCCL runtime per process (like the HIP one)
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs),
           "-L/opt/rocm/lib", "-lrccl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    # hipcc's shared link can leave per-object offload bundles (<lib>.N.hipv4-..., <lib>.N.host-...) beside the
    # library: intermediates, never loaded
    for junk in list(lib.parent.glob(lib.name + ".*.hipv4-*")) + list(lib.parent.glob(lib.name + ".*.host-*")):
        junk.unlink()
    return lib


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
