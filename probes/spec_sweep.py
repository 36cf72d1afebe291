#!/usr/bin/env python3
"""CPU-only sweep for FPSPEC v1: landmark density and hash specificity on the
music-like corpus of probes/music_eval.py, scored the way that probe scores the GPU exact lane.

Stage 1 (cached under --cache): the 1,000 indexed songs and every query clip of music_eval.py (same
seeds, same RNG order, same degradations); the peaks of every song and of every query sub-window
(app/search/exact.py SUB_WINDOWS, the engine's aid_exact_windows sample bounds) with their power,
by the C oracle at a low threshold -- a peak at threshold thr is a peak at any lower threshold with
P > thr, so one peak list serves every threshold of the sweep.

Stage 2 (per parameter set): pairing + hashing (probes/spec_sweep.c), index sort and voting
(oracle fp_index_sort / fp_query, FPSPEC 7), the reference's consensus (exact.py:220-293,
MIN_ALIGNED_HASHES 8): per category top-1, FPR and aligned-hash percentiles, as music_eval.py.

    python probes/spec_sweep.py --stage1
    python probes/spec_sweep.py --grid default
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from multiprocessing import Pool
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "probes"))

SR = 44100
HOP = 512
L5 = 5 * SR
SUB = ((0.0, 3.5), (0.75, 4.25), (1.5, 5.0))
THR_LOW = 0.25
CATS = ["clean", "noise20", "noise5", "gain-18dB", "phone", "lowpass4k", "room", "hall"]


def _olib():
    from oracle import oracle as O

    return O


def peaks_of(x):
    O = _olib()
    P = O.stft_power(x, HOP)
    pk = O.peaks(P, THR_LOW)
    p = P[pk[:, 0], pk[:, 1]] if len(pk) else np.zeros(0, np.float32)
    return pk[:, 0].astype(np.int32), pk[:, 1].astype(np.int16), p.astype(np.float32)


def _song_job(seed):
    from music_eval import song

    x = song(int(seed))
    return x, peaks_of(x)


def _windows(n):
    out = []
    for a, b in SUB:
        stop = min(b, n / SR)
        lo = min(max(int(a * SR), 0), n)
        hi = max(lo, min(int(stop * SR), n))
        out.append((lo, hi - ((hi - lo) & 1)))  # odd length -> n - 1 samples (same frames)
    return out


def _clip_job(x):
    return [peaks_of(x[lo:hi]) for lo, hi in _windows(len(x))]


def stage1(args):
    from music_eval import degrade, song

    cache = Path(args.cache)
    cache.mkdir(parents=True, exist_ok=True)
    t0 = time.perf_counter()
    seeds = np.arange(args.tracks) + 1_000_003
    songs = np.lib.format.open_memmap(cache / "songs.npy", mode="w+", dtype=np.float32, shape=(args.tracks, 30 * SR))
    pt, pk, pp, cnt = [], [], [], []
    with Pool(args.workers) as pool:
        for i, (x, (t, k, p)) in enumerate(pool.imap(_song_job, seeds, chunksize=4)):
            songs[i] = x
            pt.append(t); pk.append(k); pp.append(p); cnt.append(len(t))
            if i % 100 == 99:
                print(f"[stage1] songs {i + 1}, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
        np.savez(cache / "song_peaks.npz", t=np.concatenate(pt), k=np.concatenate(pk), p=np.concatenate(pp),
                 cnt=np.asarray(cnt, np.int64))
        songs.flush()
        # queries: music_eval.py's RNG sequence exactly
        rng = np.random.default_rng(7)
        negs = [x[:L5] for x in pool.map(song, [int(s) for s in rng.integers(10**8, 2 * 10**8, args.negatives)])]
        meta = {}
        for cat in CATS:
            pos = rng.integers(0, args.tracks, args.queries)
            starts = rng.integers(0, 25 * SR, args.queries)
            clips = [np.asarray(songs[p][s:s + L5]) for p, s in zip(pos, starts)] + negs
            clips = [degrade(c, cat, rng) for c in clips]
            wpk = pool.map(_clip_job, clips, chunksize=8)
            flat_t, flat_k, flat_p, wc = [], [], [], []
            for w3 in wpk:
                for (t, k, p) in w3:
                    flat_t.append(t); flat_k.append(k); flat_p.append(p); wc.append(len(t))
            np.savez(cache / f"q_{cat}.npz", t=np.concatenate(flat_t), k=np.concatenate(flat_k),
                     p=np.concatenate(flat_p), cnt=np.asarray(wc, np.int64), pos=pos, starts=starts)
            print(f"[stage1] {cat}, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)
        meta = {"tracks": args.tracks, "queries": args.queries, "negatives": args.negatives, "thr_low": THR_LOW}
        (cache / "meta.json").write_text(json.dumps(meta))


# ---------------------------------------------------------------- stage 2

_sw = None


def swlib():
    global _sw
    if _sw is None:
        so = Path("/tmp/aid_sweep_lib/libspecsweep.so")
        so.parent.mkdir(exist_ok=True)
        src = ROOT / "probes" / "spec_sweep.c"
        if not so.exists() or so.stat().st_mtime < src.stat().st_mtime:
            subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", str(so), str(src)], check=True)
        L = ctypes.CDLL(str(so))
        P = ctypes.c_void_p
        L.sw_hashes.restype = ctypes.c_int64
        L.sw_hashes.argtypes = [P, P, ctypes.c_int64] + [ctypes.c_int] * 7 + [P, P, ctypes.c_int64]
        L.sw_query.restype = ctypes.c_int64
        L.sw_query.argtypes = [P, ctypes.c_int64, P, P, ctypes.c_int64, ctypes.c_int, ctypes.c_int32, P,
                               ctypes.c_int64]
        _sw = L
    return _sw


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def hashes(t, k, prm):
    t = np.ascontiguousarray(t, np.int32)
    k = np.ascontiguousarray(k, np.int32)
    cap = max(1, len(t) * prm["fan"] * max(1, prm.get("triplet", 0)))
    h = np.empty(cap, np.uint32)
    t1 = np.empty(cap, np.uint32)
    n = swlib().sw_hashes(_ptr(t), _ptr(k), len(t), prm["dt_min"], prm["dt_max"], prm["df_max"], prm["fan"],
                          prm.get("triplet", 0), prm.get("tpf", 0), prm.get("apf", 0), _ptr(h), _ptr(t1), cap)
    return h[:n], t1[:n]


def select(t, k, p, prm):
    m = (p > prm["thr"]) & (k >= prm["kmin"]) & (k <= prm["kmax"])
    return t[m], k[m]


class Data:
    def __init__(self, cache):
        cache = Path(cache)
        self.meta = json.loads((cache / "meta.json").read_text())
        z = np.load(cache / "song_peaks.npz")
        self.songs = self._split(z)
        self.q = {}
        for cat in CATS:
            z = np.load(cache / f"q_{cat}.npz")
            self.q[cat] = (self._split(z), z["pos"], z["starts"])

    @staticmethod
    def _split(z):
        off = np.concatenate([[0], np.cumsum(z["cnt"])])
        t, k, p = z["t"], z["k"].astype(np.int32), z["p"]
        return [(t[a:b], k[a:b], p[a:b]) for a, b in zip(off[:-1], off[1:])]


def build_index(D, prm):
    O = _olib()
    hs, ts, tr = [], [], []
    for i, (t, k, p) in enumerate(D.songs):
        h, t1 = hashes(*select(t, k, p, prm), prm)
        hs.append(h); ts.append(t1); tr.append(np.full(len(h), i, np.uint32))
    post = np.stack([np.concatenate(hs), np.concatenate(tr), np.concatenate(ts)], axis=1).astype(np.uint32)
    post = np.ascontiguousarray(post)
    # sort by (hash, track, t): lexsort is much faster than qsort on 10M+ rows
    order = np.lexsort((post[:, 2], post[:, 1], post[:, 0]))
    return np.ascontiguousarray(post[order]), O


class SwRow(ctypes.Structure):
    _fields_ = [("score", ctypes.c_int32), ("track", ctypes.c_uint32), ("d", ctypes.c_int32)]


def query_rows(post, O, h, t1, min_match, max_rows=50, mode=0):
    rows = (SwRow * max_rows)()
    n = int(swlib().sw_query(_ptr(post), len(post), _ptr(np.ascontiguousarray(h)), _ptr(np.ascontiguousarray(t1)),
                             len(h), mode, min_match, ctypes.addressof(rows), max_rows))
    return [(r.score, r.track, r.d) for r in rows[:n]]


def consensus(wrows):
    tot, wins, starts = {}, {}, {}
    for w, rows in enumerate(wrows):
        for mc, tr, d in rows:
            tot[tr] = tot.get(tr, 0) + mc
            wins.setdefault(tr, set()).add(w)
    out = []
    for tr in tot:
        a = tot[tr] if len(wins[tr]) >= 2 else max(tot[tr] // 2, 1)
        if a >= 8:
            out.append((a, tr))
    out.sort(key=lambda x: -min(x[0] / 20, 1.0))  # stable, confidence order (exact.py:118-121)
    return out


def evaluate(D, prm, pool, cats=CATS):
    t0 = time.perf_counter()
    post, O = build_index(D, prm)
    t_idx = time.perf_counter() - t0
    res = {"params": prm, "postings": int(len(post)), "hashes_per_s": round(len(post) / (len(D.songs) * 30.0), 1)}
    nq = D.meta["queries"]
    worst = {"fpr": 0.0, "top1_clean": 1.0, "top1_degraded_min": 1.0, "unseen_max": 0}
    for cat in cats:
        wins, pos, _ = D.q[cat]
        nclip = len(wins) // 3

        def one(c):
            wr = []
            for w in range(3):
                t, k, p = wins[3 * c + w]
                h, t1 = hashes(*select(t, k, p, prm), prm)
                wr.append(query_rows(post, O, h, t1, prm["min_match"], mode=prm.get("score", 0)) if len(h) else [])
            return consensus(wr)

        out = list(pool.map(one, range(nclip)))
        hit, best, neg, fp = 0, [], [], 0
        for i, r in enumerate(out):
            top = r[0][0] if r else 0
            if i < nq:
                ok = bool(r) and r[0][1] == int(pos[i])
                hit += ok
                best.append(top if ok else 0)
            else:
                neg.append(top)
                fp += int(bool(r))
        nn = max(1, nclip - nq)
        c = {"top1": round(hit / nq, 4), "fpr": round(fp / nn, 4),
             "true_p10_p50": [int(np.percentile(best, 10)), int(np.percentile(best, 50))],
             "unseen_p50_p90_max": [int(np.percentile(neg, 50)), int(np.percentile(neg, 90)), int(max(neg))]}
        res[cat] = c
        worst["fpr"] = max(worst["fpr"], c["fpr"])
        worst["unseen_max"] = max(worst["unseen_max"], c["unseen_p50_p90_max"][2])
        if cat == "clean":
            worst["top1_clean"] = c["top1"]
        else:
            worst["top1_degraded_min"] = min(worst["top1_degraded_min"], c["top1"])
    res["worst"] = worst
    res["seconds"] = round(time.perf_counter() - t0, 1)
    res["index_s"] = round(t_idx, 1)
    return res


V0 = dict(thr=4.0, kmin=1, kmax=1023, dt_min=1, dt_max=63, df_max=127, fan=10, triplet=0, min_match=12)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cache", default="/tmp/aid_sweep")
    ap.add_argument("--stage1", action="store_true")
    ap.add_argument("--tracks", type=int, default=1000)
    ap.add_argument("--queries", type=int, default=500)
    ap.add_argument("--negatives", type=int, default=100)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--params", action="append", default=[], help="JSON overrides of V0 (repeatable)")
    ap.add_argument("--cats", default=",".join(CATS))
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    if args.stage1:
        stage1(args)
        return
    D = Data(args.cache)
    sets = [dict(V0, **json.loads(s)) for s in args.params] or [dict(V0)]
    with ThreadPoolExecutor(args.workers) as pool:
        for prm in sets:
            r = evaluate(D, prm, pool, args.cats.split(","))
            line = json.dumps(r)
            print(line, flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(line + "\n")


if __name__ == "__main__":
    main()
