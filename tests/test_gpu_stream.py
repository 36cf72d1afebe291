"""Streaming front end on the GPU: downmix bit-exact vs numpy binary32, and the
window scheduler identifying tracks of a stereo stream (config 5 shape)."""

import numpy as np
import pytest
import torch

from aidfp import synth
from aidfp.engine import Engine
from aidfp.stream import StreamIdentifier

pytestmark = pytest.mark.gpu
SR = 48000


def test_downmix_bit_exact(gpu_engine):
    rng = np.random.default_rng(0)
    for n in (1, 2, 7, 1000, 48001):
        x = rng.standard_normal((n, 2)).astype(np.float32)
        src = torch.from_numpy(x.reshape(-1)).cuda()
        dst = torch.empty(n, dtype=torch.float32, device="cuda")
        gpu_engine.downmix(src.data_ptr(), n, dst.data_ptr())
        torch.cuda.synchronize()
        ref = (x[:, 0] + x[:, 1]) * np.float32(0.5)
        assert np.array_equal(dst.cpu().numpy(), ref)


def test_stream_windows_identify_segments():
    with Engine(SR) as eng:
        from aidfp.catalog import ingest_synthetic

        ingest_synthetic(eng, np.arange(40, dtype=np.uint32), 30.0)
        seg = 30 * SR
        order = [3, 17, 29]
        L = np.concatenate([synth.synth(t, 0, seg, SR, snr_db=30.0, salt=1) for t in order])
        R = np.concatenate([synth.synth(t, 0, seg, SR, snr_db=30.0, salt=2) for t in order])
        st = np.stack([L, R], axis=1)
        sid = StreamIdentifier(eng, capacity_s=20.0)  # forces buffer compaction
        res = []
        for a in range(0, len(st), 12345):  # odd chunk sizes exercise the carry
            res += sid.push(st[a:a + 12345])
        assert len(res) == int((len(st) / SR - 5.0) // 2.5) + 1
        for r in res:
            s0 = int(round(r.start_s * SR))
            if s0 // seg == (s0 + sid.win - 1) // seg:
                assert r.best_track == order[s0 // seg]
