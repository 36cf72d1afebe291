"""Debug: per-window rows vs batched rows for one clip of tests/test_gpu_exact.py."""
import sys, uuid
sys.path[:0] = ["audio-ident_amd", "tests"]
import numpy as np
import test_gpu_exact as T
from aidfp import fingerprint as fp, exact as ex
from aidfp.engine import Engine, exact_windows
import tempfile
svc = fp.FingerprintService(tempfile.mkdtemp()); svc.persist = False
svc._engine = Engine(T.SR, device=0, min_match=4)
for i, tid in enumerate(T.IDS):
    svc.index_track(T.tr(i, 0, 30 * T.SR).astype("<f4").tobytes(), str(tid))
eng = svc._engine
cs = T.clips()
ci = int(sys.argv[1]) if len(sys.argv) > 1 else 13
x = cs[ci]
mode, wins = exact_windows(len(x), T.SR)
pieces = [x[lo:lo + ln] for lo, ln in wins if ln > 0]
print("windows", wins)
for k, p in enumerate(pieces):
    eng.extract_host([p]); r = eng.query_extracted()[0]
    print("single", k, r[r[:, 1] == 13].tolist() if len(r) else [])
eng.extract_host(pieces); rr = eng.query_extracted()
for k, r in enumerate(rr):
    print("batch3", k, r[r[:, 1] == 13].tolist() if len(r) else [])
eng.extract_host(pieces + [cs[11]]); rr = eng.query_extracted()
for k, r in enumerate(rr[:3]):
    print("batch4", k, r[r[:, 1] == 13].tolist() if len(r) else [])
print("lane", eng.exact_lane([x]))
print("lane-all", eng.exact_lane(cs)[ci])
