"""Writes tests/golden/oracle_match_v1.{npz,json}: regression vectors of FPSPEC v1 section 7 (the match scores the
DISTINCT query anchor frames of a (track, d)). Inputs: a small catalog's postings (14 synthetic v2 tracks, 8 s at
16 kHz) and query records (clean and noisy excerpts, a two-track mixture, a splice, an unseen track, a gain-reduced
clip); outputs: the oracle's rows at min_match 10 (the v1 default) and at 4, and -- to pin what v1 changed -- the
vote counts v0 would have reported for the same (track, d) rows. Run from the repo root:
python tests/golden/make_match_golden.py. NOT reference (olaf_c) outputs: none exist offline."""

import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "oracle"), str(ROOT / "audio-ident_amd")]
import oracle as O  # noqa: E402
from aidfp import synth  # noqa: E402

SR, HOP, TRACK_S = 16000, 256, 8
TRACKS = list(range(100, 114))


def raw_votes(post: np.ndarray, rec: np.ndarray, track: int, d: int) -> int:
    p = post[post[:, 1] == track]
    have = set(zip(p[:, 0].tolist(), p[:, 2].tolist()))
    h = (rec & np.uint64(0xFFFFFFFF)).astype(np.int64)
    tq = (rec >> np.uint64(32)).astype(np.int64)
    return sum((int(a), int(b) + d) in have for a, b in zip(h, tq))


def main() -> None:
    post = []
    for tr in TRACKS:
        r = O.fingerprint(synth.synth(tr, 0, TRACK_S * SR, SR), HOP)
        post.append(np.stack([(r & np.uint64(0xFFFFFFFF)).astype(np.uint32), np.full(len(r), tr, np.uint32),
                              (r >> np.uint64(32)).astype(np.uint32)], axis=1))
    post = np.concatenate(post)
    q = [
        synth.synth(101, 3 * SR, 4 * SR, SR),
        synth.synth(105, SR // 3, 3 * SR, SR, snr_db=10.0, salt=5),
        (0.5 * synth.synth(108, 2 * SR, 4 * SR, SR) + 0.5 * synth.synth(109, 4 * SR, 4 * SR, SR)).astype(np.float32),
        np.concatenate([synth.synth(110, SR, 2 * SR, SR), synth.synth(111, 5 * SR, 2 * SR, SR)]),
        synth.synth(999, 0, 4 * SR, SR, snr_db=20.0, salt=3),
        (0.05 * synth.synth(113, 0, 3 * SR, SR, snr_db=20.0, salt=8)).astype(np.float32),
    ]
    out = {"postings": post}
    meta = {"spec": "FPSPEC v1 section 7", "sr": SR, "hop": HOP, "tracks": TRACKS, "track_s": TRACK_S, "queries": []}
    for i, x in enumerate(q):
        rec = O.fingerprint(x, HOP)
        out[f"rec_{i}"] = rec
        for mm in (10, 4):
            rows = O.query(post, rec, min_match=mm, max_rows=50)
            out[f"rows_mm{mm}_{i}"] = rows
        rows4 = out[f"rows_mm4_{i}"]
        out[f"v0votes_{i}"] = np.array([raw_votes(post, rec, int(r[1]), int(r[2])) for r in rows4], np.int64)
        meta["queries"].append({"records": int(len(rec)), "rows_mm10": int(len(out[f"rows_mm10_{i}"])),
                                "rows_mm4": int(len(rows4))})
    here = Path(__file__).resolve().parent
    np.savez_compressed(here / "oracle_match_v1.npz", **out)
    (here / "oracle_match_v1.json").write_text(json.dumps(meta, indent=1))
    print(json.dumps(meta))


if __name__ == "__main__":
    main()
