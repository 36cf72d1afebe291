"""Which frames / bins of a keep-power extraction differ from the oracle (debug probe for K1 variants)."""
import sys
import numpy as np
sys.path.insert(0, "audio-ident_amd"); sys.path.insert(0, "oracle")
import oracle as O
from aidfp import synth
from aidfp.engine import Engine

SR, HOP = 44100, 512
sets = {
    "test": [(1, 441000, 0, None), (2, 100000, 12345, 20), (3, 2048, 0, None), (4, 2049, 0, None), (5, 5000, 0, None)],
    "c5only": [(5, 5000, 0, None)],
    "two": [(2, 100000, 12345, 20), (5, 5000, 0, None)],
}
for name, spec in sets.items():
    clips = [synth.synth(tr, st, n, SR, snr_db=snr, salt=7) for tr, n, st, snr in spec]
    with Engine(SR, keep_power=True) as eng:
        eng.extract_host(clips)
        for c, x in enumerate(clips):
            P = eng.power(c, len(x)); R = O.stft_power(x, HOP)
            bad = np.argwhere(P.view(np.uint32) != R.view(np.uint32))
            if len(bad):
                fr = np.unique(bad[:, 0])
                print(name, "clip", c, "frames", P.shape[0], "bad frames", fr.tolist()[:20], "n bad bins", len(bad),
                      "bins of first bad frame", bad[bad[:, 0] == fr[0], 1].tolist()[:12], flush=True)
            else:
                print(name, "clip", c, "ok", P.shape, flush=True)
