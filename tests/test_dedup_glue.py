"""Host side of the dedup drop-in (aidfp.dedup) against vectors captured from the reference
(tests/golden/ref_dedup.json, made by tests/golden/make_dedup_fixtures.py)."""

import base64
import json
from pathlib import Path

import numpy as np

from aidfp import dedup

GOLD = json.loads((Path(__file__).resolve().parent / "golden" / "ref_dedup.json").read_text())


def test_f32le_to_s16le_equals_reference():
    x = base64.b64decode(GOLD["s16"]["f32le_b64"])
    assert dedup.f32le_to_s16le(x) == base64.b64decode(GOLD["s16"]["s16le_b64"])


def test_parse_rules():
    assert dedup.parse_fingerprint("") is None
    assert dedup.parse_fingerprint("1,x,3") is None
    assert dedup.parse_fingerprint(None) is None
    assert dedup.parse_fingerprint("-1,4294967295,7").tolist() == [0xFFFFFFFF, 0xFFFFFFFF, 7]


def test_golden_file_shape():
    assert len(GOLD["similarity"]) >= 20 and len(GOLD["queries"]) >= 30
    decided = [q["result"] is not None for q in GOLD["queries"]]
    assert any(decided) and not all(decided)
    # the captured SQL bounds are the reference's duration*0.9 / duration*1.1
    for q in GOLD["queries"]:
        assert q["bounds"] == [q["duration"] * 0.9, q["duration"] * 1.1]


def test_oracle_scan_reproduces_reference_decisions():
    """oracle/fp_dedup.c (the CPU checker for big catalogs) against the reference's captured scans."""
    import oracle as O

    cat = [c for c in GOLD["catalog"] if c["fp"] is not None and c["duration"] is not None]
    arrs = [dedup.parse_fingerprint(c["fp"]) for c in cat]
    qs = [dedup.parse_fingerprint(q["fingerprint"]) for q in GOLD["queries"]]
    bi, bs = O.dedup_scan(arrs, [c["duration"] for c in cat], qs, [q["duration"] for q in GOLD["queries"]])
    for q, i, s in zip(GOLD["queries"], bi, bs):
        got = cat[i]["id"] if i >= 0 and s >= q["threshold"] else None
        assert got == q["result"]
    for pair in GOLD["similarity"]:
        a, b = dedup.parse_fingerprint(pair["fp1"]), dedup.parse_fingerprint(pair["fp2"])
        if a is None or b is None:
            continue
        assert O.lib().fp_dedup_similarity(O._ptr(a), len(a), O._ptr(b), len(b)) == pair["sim"]
