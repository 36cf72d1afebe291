#!/usr/bin/env python3
"""Extraction kernel time per audio-second by batch shape (clips x seconds) at 44.1 kHz: the headline's 256 x 10 s
steps against the catalog leg's 1,024 x 30 s batches, same generator, same box, the engine's kernel events. Each
shape is generated once and extracted repeatedly for ~--seconds of device time; the shapes are interleaved over
--rounds so clock or thermal drift shows up as a trend rather than as a shape effect. Diagnostic only.

    python probes/k1_shape_probe.py [--rounds 3] [--seconds 1.5] [--plane-rows R]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=1.5)
    ap.add_argument("--shapes", default="256x10,1024x30,256x30,1024x10")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="sync and sleep this long after every extraction call (0 = calls back to back)")
    ap.add_argument("--plane-rows", type=int, default=0,
                    help="power rows per K1 -> K2 clip group (aid_engine_force PLANE_ROWS; 0 = the engine's 3 GB default)")
    args = ap.parse_args()
    import torch

    from aidfp.engine import Engine

    sr = 44100
    torch.cuda.set_device(0)
    eng = Engine(sr, device=0)
    if args.plane_rows:
        eng.force("plane_rows", args.plane_rows)
    shapes = [tuple(int(v) for v in s.split("x")) for s in args.shapes.split(",")]
    bufs = {}
    for clips, secs in shapes:
        n = sr * secs
        pcm = torch.empty(clips * n, dtype=torch.float32, device="cuda")
        eng.synth(pcm.data_ptr(), np.arange(clips, dtype=np.uint32) + 7, np.zeros(clips, np.int64), n)
        bufs[(clips, secs)] = (pcm, np.arange(clips + 1, dtype=np.int64) * n)
    eng.profile_enable(True)
    for r in range(args.rounds):
        for shape in shapes:
            pcm, offs = bufs[shape]
            audio = shape[0] * shape[1]
            eng.extract_device(pcm.data_ptr(), offs)  # warm-up (descriptors, buffers)
            eng.sync()
            eng.profile_read(reset=True)
            reps, t0 = 0, time.perf_counter()
            while True:
                eng.extract_device(pcm.data_ptr(), offs)
                reps += 1
                if args.gap_ms > 0:
                    eng.sync()
                    time.sleep(args.gap_ms * 1e-3)
                if reps % 4 == 0:
                    eng.sync()
                    if time.perf_counter() - t0 > args.seconds:
                        break
            eng.sync()
            wall = time.perf_counter() - t0
            k = eng.profile_read(reset=True)
            per = {name: round(1e3 * ms / (reps * audio / 1000.0), 2) for name, (ms, cnt) in k.items() if cnt}
            print(json.dumps({"round": r, "clips": shape[0], "seconds": shape[1], "plane_rows": args.plane_rows,
                              "gap_ms": args.gap_ms,
                              "launches": reps,
                              "us_per_1000_audio_s": per, "wall_audio_s_per_s": round(reps * audio / wall, 1)}),
                  flush=True)
    eng.close()


if __name__ == "__main__":
    main()
