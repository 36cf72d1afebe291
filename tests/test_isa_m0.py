"""K1's add-TID LDS writes set M0 inside inline asm (csrc/stft.hip AID_TID8) and declare it clobbered; clang
does not preserve M0 across asm, so the kernel is correct only while NOTHING else in it reads or writes M0
(an LDS-DMA load, v_movrel, s_sendmsg or a compiler-placed value). This compiles stft.hip for gfx950 to device
assembly (as build_ext.py does) and fails on any M0 access outside the ;;#ASMSTART / ;;#ASMEND blocks.
CPU only: hipcc cross-compiles here."""

import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
SRC = ROOT / "audio-ident_amd" / "csrc" / "stft.hip"
HIPCC = "/opt/rocm/bin/hipcc"


def _device_asm(tmp_path) -> str:
    import sys

    sys.path.insert(0, str(ROOT / "audio-ident_amd"))
    import build_ext

    out = tmp_path / "stft.s"
    cmd = [HIPCC, *build_ext.FLAGS, *build_ext.FILE_FLAGS.get("stft.hip", []), "--cuda-device-only", "-S",
           str(SRC), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return out.read_text()


@pytest.mark.skipif(not shutil.which(HIPCC) and not Path(HIPCC).exists(), reason="hipcc not installed")
def test_m0_only_inside_add_tid_asm(tmp_path):
    text = _device_asm(tmp_path)
    inside = False
    blocks = 0
    stray = []
    m0 = re.compile(r"\bm0\b")
    for i, line in enumerate(text.splitlines()):
        s = line.strip()
        if s.startswith(";;#ASMSTART"):
            inside, blocks = True, blocks + 1
            continue
        if s.startswith(";;#ASMEND"):
            inside = False
            continue
        code = s.split(";", 1)[0]
        if m0.search(code) and not inside:
            stray.append(f"{i + 1}: {s}")
    assert blocks > 0, "no inline asm found: the add-TID writes changed, update this test"
    assert not stray, "M0 used outside the add-TID asm blocks:\n" + "\n".join(stray[:20])
