"""aidfp -- MI355X-native fingerprint extraction + match (host side).

Layers:
  * ``engine``      -- ctypes handle on libaidfp.so (HIP kernels for gfx950);
  * ``fingerprint`` -- drop-in for audio-ident-service/app/audio/fingerprint.py;
  * ``exact``       -- drop-in for audio-ident-service/app/search/exact.py glue;
  * ``synth``       -- deterministic synthetic PCM (benchmarks and tests).
"""

from ._lib import EngineError, EngineUnavailable  # noqa: F401

__all__ = ["EngineError", "EngineUnavailable"]
