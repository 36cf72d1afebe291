"""The exact-lane glue and the CSV boundary reproduce the reference's own
behaviour: vectors captured from MacPhobos/audio-ident's Python
(tests/golden/make_glue_fixtures.py -> tests/golden/ref_glue.json) are replayed
through aidfp.exact / aidfp.fingerprint. Pure host logic, no GPU."""

import asyncio
import json
import uuid
from pathlib import Path

import pytest

from aidfp import exact as ex
from aidfp import fingerprint as fp

G = json.loads((Path(__file__).resolve().parent / "golden" / "ref_glue.json").read_text())
U = [str(uuid.UUID(int=(i + 1) * 0x1111111111111111)) for i in range(6)]


def mk(d):
    return fp.OlafMatch(**d)


def asdict(m):
    return {k: getattr(m, k) for k in ("match_count", "query_start", "query_stop", "reference_path", "reference_id",
                                       "reference_start", "reference_stop")}


def cand(c):
    return {"track": str(c.track_uuid), "aligned_hashes": c.aligned_hashes, "offset": c.offset_seconds}


@pytest.mark.parametrize("case", G["parse"], ids=lambda c: repr(c["stdout"][:20]))
def test_parse_olaf_output(case):
    assert [asdict(m) for m in fp._parse_olaf_output(case["stdout"])] == case["matches"]


def test_pcm_helpers():
    for c in G["duration"]:
        assert ex.pcm_duration_sec(b"\0" * c["n_bytes"]) == c["sec"]
    for c in G["window"]:
        assert len(ex.extract_pcm_window(b"\0" * (4 * c["n_samples"]), c["start"], c["stop"])) == c["n_bytes"]
    for c in G["confidence"]:
        assert ex.normalize_confidence(c["h"]) == c["c"]


@pytest.mark.parametrize("i", range(len(G["full_clip"])))
def test_matches_to_candidates(i):
    c = G["full_clip"][i]
    assert [cand(x) for x in ex.matches_to_candidates([mk(m) for m in c["matches"]])] == c["candidates"]


@pytest.mark.parametrize("i", range(len(G["consensus"])))
def test_consensus(i):
    c = G["consensus"][i]
    got = ex.consensus_score([[mk(m) for m in w] for w in c["windows"]])
    assert [cand(x) for x in got] == c["candidates"]


def _M(cnt, path, rs):
    return fp.OlafMatch(cnt, 0.0, 3.0, path, 1, rs, rs + 3.0)


SCRIPTS = {  # the same scripted olaf_query answers the capture script fed the reference
    "strong_single": lambda i: [_M(25, U[0], 30.0)],
    "two_agree": lambda i: [_M(12, U[0], 10.0 + 0.75 * i)] if i < 2 else [],
    "mixed": lambda i: [_M(9, U[0], 1.0), _M(30, U[1], 4.0), _M(3, U[2], 2.0), _M(16, U[3], 8.0 + i)],
    "many": lambda i: [_M(10 + k, U[k % 6], float(k)) for k in range(6)],
    "missing_track": lambda i: [_M(30, U[4], 1.0), _M(28, U[5], 2.0)],
    "none": lambda i: [],
}
KNOWN = set(U[:4]) | {U[5]}


@pytest.mark.parametrize("case", G["lane"], ids=lambda c: f"{c['duration']}s-{c['script']}-{c['max_results']}")
def test_run_exact_lane(case):
    calls = []

    async def query(pcm):
        calls.append(len(pcm))
        return SCRIPTS[case["script"]](len(calls) - 1)

    async def lookup(ids):
        return {i: i for i in ids if str(i) in KNOWN}

    pcm = b"\0" * (4 * int(case["duration"] * 16000))
    res = asyncio.run(ex.run_exact_lane(pcm, case["max_results"], query=query, lookup=lookup))
    assert calls == case["calls"]
    got = [{"track": str(r.track), "confidence": r.confidence, "offset": r.offset_seconds,
            "aligned_hashes": r.aligned_hashes} for r in res]
    assert got == case["results"]


def test_olaf_error_in_subwindow_is_tolerated():
    async def query(pcm):
        raise fp.OlafError("boom")

    assert asyncio.run(ex.run_exact_lane(b"\0" * 4 * 16000 * 3, query=query)) == []
    assert asyncio.run(ex.run_exact_lane(b"\0" * 4 * 16000 * 8, query=query)) == []
