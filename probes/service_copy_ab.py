#!/usr/bin/env python3
"""A/B of the threaded host batch copy on the service leg: runs bench.py's service leg (no other legs) with
aidfp.engine._COPY_MIN set to the given number of floats (a huge value = the single-threaded copy).

    python probes/service_copy_ab.py <copy_min_floats>
"""
import runpy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "audio-ident_amd"))
import aidfp.engine as E  # noqa: E402

E._COPY_MIN = int(sys.argv[1])
sys.argv = [str(ROOT / "bench.py"), "--no-cpu", "--no-fullband", "--no-catalog", "--no-stream"]
runpy.run_path(str(ROOT / "bench.py"), run_name="__main__")
