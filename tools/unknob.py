#!/usr/bin/env python3
"""Resolve the AID_* experiment knobs of audio-ident_amd/csrc to their defaults.

Every knob was an `#ifndef AID_X / #define AID_X v / #endif` block that a -D could
override. This rewrites each source so that only the default code path is left:
  * knob definition blocks are removed;
  * `#if/#ifdef/#ifndef/#elif/#else/#endif` whose conditions name only knobs are
    evaluated and only the live branch is kept (others pass through untouched);
  * remaining uses of a knob in code are replaced by its value.
The result is checked by comparing the device ISA of the old and new builds
(tools/isa_equal.sh), so no kernel changes.

    python tools/unknob.py audio-ident_amd/csrc/*.hip audio-ident_amd/csrc/*.h audio-ident_amd/csrc/*.cpp
"""

from __future__ import annotations

import re
import sys
from pathlib import Path

KNOB = re.compile(r"\bAID_[A-Z0-9_]+\b")
# names that are ABI constants or helper macros, not knobs
KEEP_PREFIX = ("AID_OK", "AID_ERR", "AID_PCM", "AID_K_", "AID_FLAG", "AID_ABI", "AID_COMM", "AID_XCHG", "AID_TID8",
               "AID_E3A", "AID_E3B", "AID_RS_LAUNCH", "AIDFP_")


def is_knob_name(n: str) -> bool:
    return not n.startswith(KEEP_PREFIX)


def collect_defaults(files) -> dict[str, str]:
    d: dict[str, str] = {}
    for f in files:
        lines = Path(f).read_text().splitlines()
        for i, ln in enumerate(lines):
            m = re.match(r"\s*#ifndef\s+(AID_[A-Z0-9_]+)", ln)
            if not m or not is_knob_name(m.group(1)):
                continue
            name = m.group(1)
            for j in range(i + 1, min(i + 8, len(lines))):
                mm = re.match(rf"\s*#define\s+{name}\s+(.*?)\s*(//.*)?$", lines[j])
                if mm:
                    d[name] = mm.group(1)
                    break
    return d


def c_eval(expr: str, defaults: dict[str, str]):
    """Evaluate a preprocessor condition made of knobs, literals and operators; None if it names anything else."""
    e = re.sub(r"//.*", "", expr).strip()
    e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if m.group(1) in defaults else "0", e)
    e = re.sub(r"defined\s+(\w+)", lambda m: "1" if m.group(1) in defaults else "0", e)
    names = set(re.findall(r"\b[A-Za-z_]\w*\b", e))
    for n in names:
        if n in defaults:
            continue
        if n.startswith("AID_") and is_knob_name(n):  # an undefined knob (e.g. AID_K2_TWICE): 0
            continue
        return None
    e = KNOB.sub(lambda m: f"({defaults.get(m.group(0), '0')})", e)
    e = e.replace("&&", " and ").replace("||", " or ")
    e = re.sub(r"!(?!=)", " not ", e)
    try:
        return bool(eval(e, {}, {}))
    except Exception:
        return None


def process(path: Path, defaults: dict[str, str]) -> str:
    lines = path.read_text().splitlines()
    out = []
    # stack frames: ("eval", taken_any, live_now, parent_live) or ("pass", parent_live) or ("drop", parent_live)
    stack: list[tuple] = []

    def live() -> bool:
        return all(fr[-1] for fr in stack) if stack else True

    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r"#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", s)
        if not m:
            if live():
                out.append(ln)
            i += 1
            continue
        kw, rest = m.group(1), m.group(2).strip()
        if kw in ("if", "ifdef", "ifndef") and stack and stack[-1][0] == "drop":
            stack.append(("drop", False))  # nested inside a knob definition block
            i += 1
            continue
        if kw in ("if", "ifdef", "ifndef"):
            parent = live()
            name = rest.split()[0] if rest else ""
            if kw == "ifndef" and name in defaults:
                # knob definition block: drop through its #endif
                stack.append(("drop", False))
                i += 1
                continue
            if kw == "ifdef":
                cond = c_eval(f"defined({name})", defaults) if name.startswith("AID_") and is_knob_name(name) else None
            elif kw == "ifndef":
                cond = (not c_eval(f"defined({name})", defaults)) if name.startswith("AID_") and is_knob_name(name) else None
            else:
                cond = c_eval(rest, defaults)
            if cond is None:
                stack.append(["pass", parent])
                if parent:
                    out.append(ln)
            else:
                stack.append(["eval", cond, parent and cond])
            i += 1
            continue
        fr = stack[-1]
        if fr[0] == "drop":
            if kw == "endif":
                stack.pop()
            i += 1
            continue
        if fr[0] == "pass":
            if fr[1]:
                out.append(ln)
            if kw == "endif":
                stack.pop()
            i += 1
            continue
        # eval frame: [kind, taken_any, live]
        parent = all(f[-1] for f in stack[:-1]) if len(stack) > 1 else True
        if kw == "elif":
            if fr[1]:
                fr[2] = False
            else:
                c = c_eval(rest, defaults)
                if c is None:
                    raise SystemExit(f"{path}:{i + 1}: #elif on non-knob condition after knob #if")
                fr[1] = c
                fr[2] = parent and c
        elif kw == "else":
            fr[2] = parent and not fr[1]
            fr[1] = True
        elif kw == "endif":
            stack.pop()
        i += 1
    if stack:
        raise SystemExit(f"{path}: unbalanced conditionals")
    text = "\n".join(out) + "\n"

    # knob uses left in code -> their values
    def sub(m):
        n = m.group(0)
        if n in defaults:
            return defaults[n]
        return n

    text = KNOB.sub(sub, text)
    return text


def main(argv):
    files = [Path(a) for a in argv]
    defaults = collect_defaults(files)
    for f in files:
        new = process(f, defaults)
        if new != f.read_text():
            f.write_text(new)
            print("rewrote", f)
    print(f"{len(defaults)} knobs resolved")


if __name__ == "__main__":
    main(sys.argv[1:])
