"""Capture the reference's exact-lane glue behaviour as JSON vectors.

Runs ONLY in the build container (it imports the reference Python from
/root/reference, read-only; nothing of it is copied into this repo or shipped
to the GPU box). Output: tests/golden/ref_glue.json -- inputs and outputs of
  app/audio/fingerprint.py  _parse_olaf_output            (:273-301)
  app/search/exact.py       _pcm_duration_sec             (:361-371)
                            _extract_pcm_window           (:374-399)
                            _normalize_confidence         (:340-353)
                            _matches_to_candidates        (:296-332)
                            _consensus_score              (:220-293)
                            run_exact_lane (olaf_query + DB patched) (:70-124)
Import shims: enum.StrEnum for Python 3.10, a pydantic_settings
stand-in module, and a stub app.db.session (the module only builds an engine).

Run: python tests/golden/make_glue_fixtures.py
"""

from __future__ import annotations

import asyncio
import enum
import json
import struct
import sys
import types
import uuid
from pathlib import Path
from unittest.mock import patch

REF = Path("/root/reference/audio-ident-service")
OUT = Path(__file__).resolve().parent / "ref_glue.json"


def _shims() -> None:
    if not hasattr(enum, "StrEnum"):
        class StrEnum(str, enum.Enum):
            pass

        enum.StrEnum = StrEnum
    import pydantic

    ps = types.ModuleType("pydantic_settings")

    class BaseSettings(pydantic.BaseModel):
        model_config = pydantic.ConfigDict(extra="ignore")

    ps.BaseSettings = BaseSettings
    ps.SettingsConfigDict = lambda **kw: dict(kw)
    sys.modules["pydantic_settings"] = ps
    sess = types.ModuleType("app.db.session")
    sess.async_session_factory = None
    sys.modules["app.db.session"] = sess
    sys.path.insert(0, str(REF))


def match_dict(m) -> dict:
    return {k: getattr(m, k) for k in ("match_count", "query_start", "query_stop", "reference_path", "reference_id",
                                       "reference_start", "reference_stop")}


U = [str(uuid.UUID(int=(i + 1) * 0x1111111111111111)) for i in range(6)]


def main() -> None:
    _shims()
    from app.audio import fingerprint as fp
    from app.search import exact as ex

    out: dict = {"source": "MacPhobos/audio-ident reference, captured by tests/golden/make_glue_fixtures.py"}

    # ---- CSV parsing
    csvs = [
        "",
        "   \n  \n",
        "42, 0.5, 3.2, 12345678-1234-5678-1234-567812345678, 1001, 10.0, 12.7\n15, 1.0, 2.5, t2, 1002, 5.0, 6.5\n",
        "not,enough,fields\n42, 0.5, 3.2, track, 1001, 10.0, 12.7\n",
        "42; 0.5; 3.2; my-track; 1001; 10.0; 12.7",
        "abc, 0.5, 3.2, track, 1001, 10.0, 12.7",
        "5, 0.0, 1.0, a, 1, 0.0, 1.0\n99, 0.0, 1.0, b, 2, 0.0, 1.0\n20, 0.0, 1.0, c, 3, 0.0, 1.0\n7, 0, 1, d, 4, 0, 1\n",
        "7, 0, 1, d, 4, 0, 1, extra, fields\n7, 0.25, 1.5, e, 5, 2, 3\n",
        "1,2,3,x,5,6\n3,1e-3,2.5e1,y,9,1.5,2.5\n  8 , 1 , 2 , spaced , 3 , 4 , 5  \n",
    ]
    out["parse"] = [{"stdout": s, "matches": [match_dict(m) for m in fp._parse_olaf_output(s)]} for s in csvs]

    # ---- PCM helpers
    out["duration"] = [{"n_bytes": n, "sec": ex._pcm_duration_sec(b"\0" * n)} for n in (0, 4, 64000, 64004, 320000, 3)]
    wins = []
    for n_samp in (0, 16000, 56000, 80000, 96000, 12345):
        pcm = b"\0" * (4 * n_samp)
        for a, b in ((0.0, 3.5), (0.75, 4.25), (1.5, 5.0), (0.0, 1.0), (5.0, 9.0), (2.0, 1.0), (0.1234, 0.5678)):
            wins.append({"n_samples": n_samp, "start": a, "stop": b, "n_bytes": len(ex._extract_pcm_window(pcm, a, b))})
    out["window"] = wins
    out["confidence"] = [{"h": h, "c": ex._normalize_confidence(h)} for h in range(-5, 46)]

    # ---- aggregation / consensus
    def M(cnt, path, rs, qs=0.0, rid=1):
        return fp.OlafMatch(match_count=cnt, query_start=qs, query_stop=qs + 3.0, reference_path=path,
                            reference_id=rid, reference_start=rs, reference_stop=rs + 3.0)

    cand = lambda c: {"track": str(c.track_uuid), "aligned_hashes": c.aligned_hashes, "offset": c.offset_seconds}
    full_cases = [
        [],
        [M(25, U[0], 30.0)],
        [M(12, U[0], 10.0), M(10, U[0], 10.5), M(9, U[1], 3.0)],
        [M(5, "not-a-uuid", 1.0), M(7, U[2], 2.0), M(3, f"  {U[2]} ", 4.0), M(1, U[2], 9.0)],
    ]
    out["full_clip"] = [{"matches": [match_dict(m) for m in ms], "candidates": [cand(c) for c in ex._matches_to_candidates(ms)]}
                        for ms in full_cases]
    win_cases = [
        [[], [], []],
        [[M(12, U[0], 10.0)], [M(10, U[0], 10.75)], []],
        [[M(10, U[0], 10.0)], [M(8, U[0], 10.75)], [M(12, U[0], 11.5)]],
        [[M(20, U[0], 10.0)], [], []],
        [[M(1, U[1], 4.0)], [], []],
        [[M(9, U[0], 1.0)], [M(14, U[1], 2.0)], [M(11, U[2], 3.0)]],
        [[M(9, U[0], 1.0), M(4, U[0], 7.0)], [M(14, U[1], 2.0)], [M(11, U[0], 3.0), M(2, "x", 0.0)]],
        [[M(3, U[3], 5.0), M(3, U[4], 5.0)], [M(6, U[4], 5.5)], [M(2, U[3], 6.0), M(8, U[5], 0.5)]],
    ]
    out["consensus"] = [{"windows": [[match_dict(m) for m in w] for w in ws],
                         "candidates": [cand(c) for c in ex._consensus_score(ws)]} for ws in win_cases]

    # ---- run_exact_lane end to end (olaf_query and the DB patched)
    lanes = []
    scripts = {
        "strong_single": lambda i, n: [M(25, U[0], 30.0)],
        "two_agree": lambda i, n: [M(12, U[0], 10.0 + 0.75 * i)] if i < 2 else [],
        "mixed": lambda i, n: [M(9, U[0], 1.0), M(30, U[1], 4.0), M(3, U[2], 2.0), M(16, U[3], 8.0 + i)],
        "many": lambda i, n: [M(10 + k, U[k % 6], float(k)) for k in range(6)],
        "missing_track": lambda i, n: [M(30, U[4], 1.0), M(28, U[5], 2.0)],
        "none": lambda i, n: [],
    }
    known = set(U[:4]) | {U[5]}
    for dur in (0.0, 1.0, 2.0, 3.5, 4.0, 5.0, 5.01, 6.0, 10.0):
        for name, fn in scripts.items():
            calls: list[int] = []

            async def fake_query(pcm: bytes, _fn=fn, _calls=calls):
                _calls.append(len(pcm))
                return _fn(len(_calls) - 1, len(pcm))

            async def fake_lookup(session, ids):
                return {i: types.SimpleNamespace(id=i, title="t", artist=None, album=None, duration_seconds=60.0,
                                                 ingested_at="2025-01-15T12:00:00Z") for i in ids if str(i) in known}

            def info(track):
                return {"id": str(track.id)}

            pcm = struct.pack(f"<{int(dur * 16000)}f", *([0.0] * int(dur * 16000)))
            with patch.object(ex, "olaf_query", fake_query), patch.object(ex, "get_tracks_by_ids", fake_lookup), \
                    patch.object(ex, "_track_to_info", lambda t: ex.TrackInfo(id=t.id, title="t", duration_seconds=60.0,
                                                                          ingested_at="2025-01-15T12:00:00Z")):
                for mr in (10, 2):
                    calls.clear()
                    res = asyncio.run(ex.run_exact_lane(pcm, mr, session=object()))
                    lanes.append({"duration": dur, "script": name, "max_results": mr, "calls": list(calls),
                                  "results": [{"track": str(r.track.id), "confidence": r.confidence,
                                               "offset": r.offset_seconds, "aligned_hashes": r.aligned_hashes}
                                              for r in res]})
    out["lane"] = lanes
    OUT.write_text(json.dumps(out, indent=1, sort_keys=True))
    print(f"wrote {OUT} ({len(lanes)} lane cases)")


if __name__ == "__main__":
    main()
