#!/usr/bin/env python3
"""bench.py -- fingerprint-extraction throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): a batch of 256 x 10 s
44.1 kHz mono synthetic clips, resident in HBM (generated on the device by
aid_synth). One step = one pass of K1 stft_power -> K2 peak_pick -> K3
landmark_hash (count + write) over the whole batch through the C ABI.

N GPUs: one process per GPU (torch.distributed, RCCL backend), each rank
fingerprints its own 256-clip batch (extraction shards by clip, no data-path
collective: weak scaling). value = audio-seconds of all ranks / max-rank time.

Roofline: the dominant kernel's algorithmic HBM bytes per launch (DESIGN.md
"Roofline") / its mean launch time from HIP events recorded on the launch
stream during the timed region, against 8.0 TB/s. cpu_baseline: the C oracle
(oracle/fp_oracle.c, bit-exact restatement) on rank 0 at N=1 over a bounded
sample of the same clips.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))

METRIC = "audio-seconds fingerprinted/sec/GPU; landmark-hash bit-exact vs CPU ref"
SR = 44100
CLIPS = 256
CLIP_S = 10
HBM_PEAK_GBS = 8000.0


def algorithmic_bytes(frames: int, samples: int) -> dict:
    """Per-launch algorithmic HBM bytes of each extraction kernel."""
    return {
        # K1 reads every PCM sample once, writes 1024 fp32 bins per frame
        "stft_power": 4 * samples + 4 * 1024 * frames,
        # K2 reads the power plane once, writes a 128-byte peak mask per frame
        "peak_pick": 4 * 1024 * frames + 128 * frames,
    }


def load_pmc(kernel: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if present."""
    for f in sorted((ROOT / "profiles").glob("pmc_*.json"), reverse=True):
        try:
            d = json.loads(f.read_text())
            k = d.get("kernels", {}).get(kernel)
            if k and k.get("hbm_bytes_per_launch"):
                return float(k["hbm_bytes_per_launch"]), f.name
        except Exception:
            continue
    return None, None


def parity(eng, host_pcm: np.ndarray, ref=None) -> dict:
    """Hashes of the bench batch (left by the last step) against the C oracle, bit for bit.

    `ref` = the oracle's records for the first len(ref) clips when the cpu_baseline leg already
    computed them; otherwise the oracle runs here on the first 8 clips."""
    if ref is None:
        sys.path.insert(0, str(ROOT / "oracle"))
        import oracle as O  # checker only

        ref = O.fingerprint_batch(host_pcm[:8], 512, threads=min(8, os.cpu_count() or 1))
    bad = [c for c in range(len(ref)) if not np.array_equal(eng.hashes(c), ref[c])]
    return {"clips": len(ref), "hashes": int(sum(len(r) for r in ref)), "bit_exact": not bad,
            "mismatched_clips": bad[:8], "oracle": "oracle/fp_oracle.c"}


def cpu_baseline(host_pcm: np.ndarray, min_s: float = 6.0) -> tuple[dict, list]:
    """The C oracle on the host cores over the bench batch: passes of all 256 clips on `threads` threads until
    `min_s` seconds have elapsed (>= 1 pass; ~10 s of CPU work with the single-thread leg), then 64 clips on
    one thread. Returns the oracle's records of the batch (for the parity check) and the baseline dict."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as O  # checker / CPU baseline only

    threads = min(16, os.cpu_count() or 1)
    sample = host_pcm[: min(len(host_pcm), 256)]
    O.fingerprint_batch(sample[:2], 512, threads=1)  # warm (tables)
    passes = 0
    t = time.perf_counter()
    while True:
        ref = O.fingerprint_batch(sample, 512, threads=threads)
        passes += 1
        dt_mt = time.perf_counter() - t
        if dt_mt >= min_s:
            break
    one = sample[:64]
    t = time.perf_counter()
    O.fingerprint_batch(one, 512, threads=1)
    dt_1 = time.perf_counter() - t
    audio_mt = passes * sample.shape[0] * sample.shape[1] / SR
    audio_1 = one.shape[0] * one.shape[1] / SR
    return ref, {
        "value": round(audio_mt / dt_mt, 1),
        "unit": "audio-s/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{passes} pass(es) over the {sample.shape[0]} x {CLIP_S} s clips of the same batch through "
                  f"oracle/fp_oracle.c (bit-exact C restatement, -O2) on {threads} host threads ({dt_mt:.1f} s); "
                  f"single-thread {audio_1 / dt_1:.1f} audio-s/s over {one.shape[0]} clips ({dt_1:.1f} s)",
    }


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--settle", type=float, default=0.1,
                    help="seconds of untimed steps after the warmup steps (GPU clock ramp); 0 = none")
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        # AIDFP_BENCH_BACKEND=gloo: rehearsal of the N-rank path on fewer GPUs than ranks (ranks share
        # devices round-robin; RCCL refuses two ranks on one GPU). The driver's runs use RCCL, one GPU each.
        backend = os.environ.get("AIDFP_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            torch.cuda.set_device(local % torch.cuda.device_count())
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)

    from aidfp.engine import Engine

    eng = Engine(SR, device=torch.cuda.current_device())
    n = SR * CLIP_S
    pcm = torch.empty(CLIPS * n, dtype=torch.float32, device="cuda")
    tracks = np.arange(CLIPS, dtype=np.uint32) + np.uint32(rank * CLIPS)
    eng.synth(pcm.data_ptr(), tracks, np.zeros(CLIPS, np.int64), n)
    offs = np.arange(CLIPS + 1, dtype=np.int64) * n
    stream = torch.cuda.current_stream().cuda_stream
    frames = CLIPS * eng.num_frames(n)

    for _ in range(max(0, args.warmup)):
        eng.extract_device(pcm.data_ptr(), offs, stream)
    torch.cuda.synchronize()
    # settle: keep stepping (untimed) until the GPU has been busy for SETTLE_S. An idle MI355X
    # needs ~25 ms of load to reach its steady clocks: the first 20 steps after start-up (or after
    # 0.5 s idle) ran K1 at 0.345 ms against 0.303 ms steady (probes/ramp_probe.py)
    settle_steps = 0
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle:
        for _ in range(10):
            eng.extract_device(pcm.data_ptr(), offs, stream)
        settle_steps += 10
        torch.cuda.synchronize()
    hashes_per_step = int(eng.counts().sum())

    # events inside the timed region on K1 (stft_power, the dominant kernel) only: every timed launch
    # carries two dispatch-attached events, ~6 us of end-of-kernel work per launch on MI355X
    # (probes/prof_overhead.py: 4.72 M audio-s/s with K1-K3 timed, 4.82 M with K1 only, 4.86 M with
    # none). The per-kernel breakdown comes from an untimed pass after the timed region.
    eng.profile_select([0])
    eng.profile_enable(True)
    eng.profile_read(reset=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.extract_device(pcm.data_ptr(), offs, stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = eng.profile_read(reset=True)
    # untimed breakdown pass: every extraction kernel gets events
    eng.profile_select(None)
    for _ in range(max(1, min(args.steps, 20))):
        eng.extract_device(pcm.data_ptr(), offs, stream)
    torch.cuda.synchronize()
    prof_all = eng.profile_read(reset=True)
    eng.profile_enable(False)

    if dist:
        on_dev = dist.get_backend() == "nccl"
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    audio_s = world * CLIPS * CLIP_S * args.steps
    value = audio_s / elapsed

    live = {k: {"ms_per_launch": (ms / cnt if cnt else None), "launches": cnt} for k, (ms, cnt) in prof.items() if cnt}
    kern = {k: {"ms_per_launch": (ms / cnt if cnt else None), "launches": cnt, "pass": "untimed breakdown"}
            for k, (ms, cnt) in prof_all.items() if cnt}
    for k, v in live.items():  # the timed region's own events win where they exist
        kern[k] = {**v, "pass": "timed region"}
    alg = algorithmic_bytes(frames, CLIPS * n)
    # dominant kernel from the breakdown pass; its duration from the timed region when it was timed there
    dom = max(("stft_power", "peak_pick"),
              key=lambda k: prof_all[k][0] / prof_all[k][1] if k in prof_all and prof_all[k][1] else 0.0)
    dom_ms = kern[dom]["ms_per_launch"]
    achieved = alg[dom] / (dom_ms * 1e-3) / 1e9
    pmc, pmc_src = load_pmc(dom)
    roofline = {
        "kernel": dom,
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": pmc,
        "algorithmic_bytes_per_launch": alg[dom],
        "traffic_source": pmc_src,
        "duration_source": kern[dom]["pass"],
        "extraction_kernels_ms_per_step": round(sum(v["ms_per_launch"] for v in kern.values() if v["ms_per_launch"]), 4),
        # the whole step against the same staged-dataflow accounting (K1 + K2 bytes of SURVEY 8(d); K3's
        # mask reads and record writes are < 1 % and left out): how far the pipeline is from streaming
        "step_staged_bytes": alg["stft_power"] + alg["peak_pick"],
        "step_achieved": round((alg["stft_power"] + alg["peak_pick"]) / (elapsed / args.steps) / 1e9, 1),
        "note": "achieved = SURVEY 8(d) staged-dataflow bytes (PCM + the full power plane); K1 stores only hot "
                "64-bin blocks and K2 reads only those, so the PMC traffic can be below the algorithmic bytes",
    }

    cpu = par = None
    if rank == 0:
        host = pcm.view(CLIPS, n).cpu().numpy()
        ref = None
        if world == 1 and not args.no_cpu:
            ref, cpu = cpu_baseline(host)
        # untimed: the batch's hashes (from the last step) against the oracle's
        par = parity(eng, host, ref)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "audio-s/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_steps": settle_steps,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (aid_synth: seed-42 integer-exact partials + noise, generated in HBM)",
            "config": {
                "workload": "BASELINE configs[1]: 256 x 10 s 44.1 kHz mono clips, fingerprint extraction per GPU",
                "clips_per_gpu": CLIPS,
                "clip_seconds": CLIP_S,
                "sample_rate": SR,
                "n_fft": 2048,
                "hop": eng.hop,
                "parallelism": f"replicas x{world} (clip-sharded, no collective)",
            },
            "realtime_factor_per_gpu": round(value / world, 1),
            "hashes_per_step_per_gpu": hashes_per_step,
            "kernels": kern,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": par,
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()
    return 0 if par is None or par["bit_exact"] else 1


if __name__ == "__main__":
    sys.exit(main())
