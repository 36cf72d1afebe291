"""PCIe-inclusive extraction rate: the bench batch (256 x 10 s at 44.1 kHz) handed to aid_extract as
HOST memory -- pageable (numpy, what the olaf_c adapter passes) and pinned -- against the same batch resident in HBM
(the bench's `value`). Every variant runs the same K1-K3; host variants add the H2D copy of 451.6 MB per step.

usage: python probes/pcie_probe.py [--steps N]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "audio-ident_amd"))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import ctypes

    import torch
    from aidfp._lib import check
    from aidfp.engine import AID_PCM_HOST, Engine

    SR, CLIPS, SEC = 44100, 256, 10
    n = SR * SEC
    eng = Engine(SR)
    pcm = torch.empty(CLIPS * n, dtype=torch.float32, device="cuda")
    eng.synth(pcm.data_ptr(), np.arange(CLIPS, dtype=np.uint32) + 1, np.zeros(CLIPS, np.int64), n)
    offs = np.arange(CLIPS + 1, dtype=np.int64) * n
    torch.cuda.synchronize()
    pinned = pcm.cpu().pin_memory()
    pageable = pcm.cpu().numpy().copy()
    audio = CLIPS * SEC
    out = {"batch": f"{CLIPS} x {SEC} s at {SR} Hz", "bytes_per_step": int(pcm.numel() * 4), "steps": args.steps}

    def timed(fn) -> float:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / args.steps

    def host(ptr):
        return lambda: check(eng._lib.aid_extract(eng._h, ctypes.c_void_p(ptr), offs.ctypes.data_as(ctypes.c_void_p),
                                                  CLIPS, AID_PCM_HOST, None))

    for name, fn in (("device", lambda: eng.extract_device(pcm.data_ptr(), offs)),
                     ("host_pinned", host(pinned.data_ptr())),
                     ("host_pageable", host(pageable.ctypes.data))):
        s = timed(fn)
        out[name] = {"ms_per_step": round(s * 1e3, 3), "audio_s_per_s": round(audio / s, 1),
                     "h2d_gbs": None if name == "device" else round(out["bytes_per_step"] / s / 1e9, 1)}
    # the records of the last step agree across the three inputs
    eng.extract_device(pcm.data_ptr(), offs)
    ref = [eng.hashes(c) for c in range(0, CLIPS, 37)]
    host(pageable.ctypes.data)()
    got = [eng.hashes(c) for c in range(0, CLIPS, 37)]
    out["records_equal"] = all(np.array_equal(a, b) for a, b in zip(ref, got))
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
