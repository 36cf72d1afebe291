#!/usr/bin/env python3
"""Where K2's wave-cycles go, by s_memtime segments (diagnostic build, AID_K2_STAMPS).

    python probes/k2_stamps_probe.py [--steps 20]

Loads the diagnostic copy of the library (audio-ident_amd/build/k2stamps/libaidfp.so, built by
build_ext.build(variant="k2stamps", defines=("AID_K2_STAMPS",))), runs the bench batch (256 x 10 s, band-limited and
full-band), and prints the share of a surviving K2 wave's life spent at the first barrier of its 4-row steps (waiting
for the other waves of its workgroup to finish the previous rows), with the diagnostic build's own K2 time beside the
product's to show what the stamps cost. Prints one JSON line."""
import argparse
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
VARIANT = ROOT / "audio-ident_amd" / "build" / "k2stamps" / "libaidfp.so"
os.environ["AIDFP_LIB"] = str(VARIANT)
sys.path.insert(0, str(ROOT / "audio-ident_amd"))

SEGS = ["barrier_before_staging"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from aidfp import _lib
    from aidfp.engine import Engine

    lib = _lib.load()
    fn = lib.aid_diag_k2_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    torch.cuda.set_device(0)
    eng = Engine(44100, device=0)
    n, clips = 441000, 256
    pcm = torch.empty(clips * n, dtype=torch.float32, device="cuda")
    offs = np.arange(clips + 1, dtype=np.int64) * n
    out = {"library": str(VARIANT.relative_to(ROOT)), "steps": args.steps}
    buf = np.zeros(8, dtype=np.uint64)
    for name, fmax in (("bench_data", 8000), ("full_band", 20000)):
        eng.synth(pcm.data_ptr(), np.arange(clips, dtype=np.uint32), np.zeros(clips, np.int64), n, fmax_hz=fmax)
        for _ in range(30):  # warm + clocks + the adaptive strip sizing settles
            eng.extract_device(pcm.data_ptr(), offs)
        torch.cuda.synchronize()
        fn(buf.ctypes.data, 1)
        eng.profile_select([1])
        eng.profile_enable(True)
        eng.profile_read(reset=True)
        for _ in range(args.steps):
            eng.extract_device(pcm.data_ptr(), offs)
        torch.cuda.synchronize()
        prof = eng.profile_read(reset=True)
        eng.profile_enable(False)
        fn(buf.ctypes.data, 1)
        seg = buf[:1].astype(np.float64)
        life = float(buf[6])
        waves = int(buf[5]) // args.steps
        out[name] = {"k2_ms": round(prof["peak_pick"][0] / max(1, prof["peak_pick"][1]), 4),
                     "surviving_waves_per_launch": waves, "exiting_waves_per_launch": int(buf[7]) // args.steps,
                     "mean_wave_life_cycles": round(life / max(1, int(buf[5])), 1),
                     "share_of_wave_life": {k: round(float(v) / life, 4) for k, v in zip(SEGS, seg)}}
        print(json.dumps({name: out[name]}), file=sys.stderr, flush=True)
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
