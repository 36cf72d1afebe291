import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "audio-ident_amd", ROOT / "oracle", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libaidfp.so")


@pytest.fixture(scope="session")
def gpu_engine():
    """One engine per session (44.1 kHz); GPU tests share it (one process on the card)."""
    from aidfp.engine import Engine

    eng = Engine(44100)
    yield eng
    eng.close()
