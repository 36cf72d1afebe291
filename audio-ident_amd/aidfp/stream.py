"""Continuous identification of a 48 kHz stereo stream (BASELINE config 5).

The reference has no streaming path: its UI records 48 kHz mono clips
(audio-ident-ui AudioRecorder.svelte:86-106), ffmpeg downmixes/resamples them
(app/audio/decode.py:41-60) and each clip is one exact-lane query. Here a
stream is consumed in chunks: every chunk of interleaved stereo is downmixed on
the GPU (aid_downmix) into a device buffer of mono PCM, and every `hop_s` of new
audio completes one `window_s` window (50 % overlap by default). All windows
completed by a push are fingerprinted and matched in one batched engine call
(K1-K3 + K5) against an index built at the stream's sample rate.
"""

from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class WindowResult:
    start_s: float        # window start in stream time
    rows: np.ndarray      # [r, 5] int64 (match_count, track, d, tq_min, tq_max)

    @property
    def best_track(self):
        return int(self.rows[0, 1]) if len(self.rows) else None


class StreamIdentifier:
    def __init__(self, engine, window_s: float = 5.0, hop_s: float = 2.5, capacity_s: float = 120.0):
        import torch

        self.eng = engine
        self.sr = engine.sample_rate
        self.win = int(round(window_s * self.sr)) & ~1
        self.hop = int(round(hop_s * self.sr)) & ~1
        cap = max(int(capacity_s * self.sr), 4 * self.win) & ~1
        self.mono = torch.zeros(cap, dtype=torch.float32, device="cuda")
        self.stage = torch.empty(0, dtype=torch.float32, device="cuda")
        self.win_buf = torch.empty(0, dtype=torch.float32, device="cuda")
        self.carry = np.zeros((0, 2), dtype=np.float32)  # odd trailing frame kept for the next push
        self.filled = 0      # valid samples in self.mono (always even)
        self.base = 0        # stream sample index of self.mono[0]
        self.next_start = 0  # stream sample index of the next window

    def push(self, stereo: np.ndarray) -> list[WindowResult]:
        """stereo: [n, 2] float32 host chunk. Returns the windows this chunk completed."""
        import torch

        x = np.ascontiguousarray(stereo, dtype=np.float32).reshape(-1, 2)
        if len(self.carry):
            x = np.concatenate([self.carry, x])
        n = len(x) & ~1
        self.carry = x[n:].copy()
        x = x[:n]
        if n == 0:
            return []
        if self.filled + n > self.mono.numel():  # compact: keep what pending windows still need
            drop = (self.next_start - self.base) & ~1
            keep = self.filled - drop
            if keep + n > self.mono.numel():
                raise ValueError("chunk larger than the stream buffer")
            self.mono[:keep] = self.mono[drop:self.filled].clone()
            self.base += drop
            self.filled = keep
        if self.stage.numel() < 2 * n:
            self.stage = torch.empty(2 * n, dtype=torch.float32, device="cuda")
        self.stage[: 2 * n].copy_(torch.from_numpy(x.reshape(-1)))
        s = torch.cuda.current_stream().cuda_stream
        self.eng.downmix(self.stage.data_ptr(), n, self.mono.data_ptr() + 4 * self.filled, s)
        self.filled += n
        starts = []
        while self.next_start + self.win <= self.base + self.filled:
            starts.append(self.next_start)
            self.next_start += self.hop
        if not starts:
            return []
        # overlapping windows -> one contiguous clip each (device copies), one batched call
        k = len(starts)
        if self.win_buf.numel() < k * self.win:
            self.win_buf = torch.empty(k * self.win, dtype=torch.float32, device="cuda")
        for i, st in enumerate(starts):
            r = st - self.base
            self.win_buf[i * self.win:(i + 1) * self.win] = self.mono[r:r + self.win]
        self.eng.extract_device(self.win_buf.data_ptr(), np.arange(k + 1, dtype=np.int64) * self.win, s)
        rows = self.eng.query_extracted()
        return [WindowResult(st / self.sr, r) for st, r in zip(starts, rows)]
