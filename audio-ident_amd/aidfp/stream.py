"""Continuous identification of a stereo stream (BASELINE config 5).

The reference has no streaming path: its UI records 48 kHz mono clips
(audio-ident-ui AudioRecorder.svelte:86-106), ffmpeg downmixes/resamples them
(app/audio/decode.py:41-60) and each clip is one exact-lane query. Here a
stream is consumed in chunks, and every chunk of interleaved stereo becomes mono
PCM at the INDEX's sample rate in a device buffer:
  * same rate: downmix on the GPU (aid_downmix);
  * other rate: downmix + polyphase resampling on the GPU (aid_resample_range, FPSPEC 8).
    The raw stereo history the filter still needs stays on the device, and each push
    produces exactly the outputs whose filter window is complete, so the chunked
    result equals resampling the whole stream at once (tests/test_gpu_resample.py).
Every `hop_s` of new audio completes one `window_s` window (50 % overlap by default).
All windows completed by a push are fingerprinted and matched in one batched
engine call (K1-K3 + K5) against the index.
"""

from __future__ import annotations

import time
from dataclasses import dataclass

import numpy as np


@dataclass(slots=True)  # 256 per push of a full stream bank: slots make each construction cheaper
class WindowResult:
    start_s: float        # window start in stream time
    rows: np.ndarray      # [r, 5] int64 (match_count, track, d, tq_min, tq_max)

    @property
    def best_track(self):
        return int(self.rows[0, 1]) if len(self.rows) else None


class StreamIdentifier:
    def __init__(self, engine, window_s: float = 5.0, hop_s: float = 2.5, capacity_s: float = 120.0,
                 stream_sr: int | None = None):
        import torch

        self.eng = engine
        self.sr = engine.sample_rate               # index rate = rate of the mono buffer
        self.stream_sr = int(stream_sr or self.sr)
        self.win = int(round(window_s * self.sr)) & ~1
        self.hop = int(round(hop_s * self.sr)) & ~1
        cap = max(int(capacity_s * self.sr), 4 * self.win) & ~1
        self.mono = torch.zeros(cap, dtype=torch.float32, device="cuda")
        self.stage = torch.empty(0, dtype=torch.float32, device="cuda")
        self.win_buf = torch.empty(0, dtype=torch.float32, device="cuda")
        self.carry = np.zeros((0, 2), dtype=np.float32)  # odd trailing frame kept for the next push
        self._pin = None     # pinned host staging of a chunk (asynchronous H2D, about twice the pageable rate)
        self._pin_ev = None  # recorded after the copy out of _pin: the next push waits for it before refilling
        self.filled = 0      # valid samples in self.mono
        self.base = 0        # stream sample index (index rate) of self.mono[0]; always even
        self.next_start = 0  # stream sample index of the next window
        self.resampling = self.stream_sr != self.sr
        if self.resampling:
            self.up, self.down, self.hl, self.J = engine.resample_plan(self.stream_sr, self.sr)
            cap_in = max(int(capacity_s * self.stream_sr), 4 * int(window_s * self.stream_sr))
            self.raw = torch.zeros(2 * cap_in, dtype=torch.float32, device="cuda")  # interleaved stereo
            self.raw_base = 0    # stream frame index (stream rate) of raw[0]
            self.raw_filled = 0  # frames held
            self.n_in = 0        # frames received
            self.m_next = 0      # next output sample (index rate) to produce

    def _h2d(self, dst, x: np.ndarray) -> None:
        """dst[:n] = x (flat float32) through the pinned staging buffer, asynchronously on the current stream."""
        import torch

        n = x.size
        if self._pin_ev is not None:
            self._pin_ev.synchronize()  # the previous chunk has left the staging buffer
        if self._pin is None or self._pin.numel() < n:
            self._pin = torch.empty(n, dtype=torch.float32).pin_memory()
            self._pin_ev = torch.cuda.Event()
        self._pin.numpy()[:n] = x
        dst[:n].copy_(self._pin[:n], non_blocking=True)
        self._pin_ev.record()

    # -- mono buffer (index rate) --
    def _reserve_mono(self, n: int) -> None:
        if self.filled + n > self.mono.numel():  # compact: keep what pending windows still need
            drop = (self.next_start - self.base) & ~1
            keep = self.filled - drop
            if keep + n > self.mono.numel():
                raise ValueError("chunk larger than the stream buffer")
            self.mono[:keep] = self.mono[drop:self.filled].clone()
            self.base += drop
            self.filled = keep

    def _push_same_rate(self, x: np.ndarray, s: int) -> None:
        import torch

        if len(self.carry):
            x = np.concatenate([self.carry, x])
        n = len(x) & ~1
        self.carry = x[n:].copy()
        x = x[:n]
        if n == 0:
            return
        self._reserve_mono(n)
        if self.stage.numel() < 2 * n:
            self.stage = torch.empty(2 * n, dtype=torch.float32, device="cuda")
        self._h2d(self.stage, x.reshape(-1))
        self.eng.downmix(self.stage.data_ptr(), n, self.mono.data_ptr() + 4 * self.filled, s)
        self.filled += n

    def _push_resampled(self, x: np.ndarray, s: int) -> None:
        import torch

        n = len(x)
        if n == 0:
            return
        cap_in = self.raw.numel() // 2
        if self.raw_filled + n > cap_in:  # compact: keep the input the next output still reads
            need = max(self.raw_base, (self.m_next * self.down + self.hl) // self.up - (self.J - 1))
            drop = need - self.raw_base
            keep = self.raw_filled - drop
            if keep + n > cap_in:
                raise ValueError("chunk larger than the stream buffer")
            self.raw[: 2 * keep] = self.raw[2 * drop: 2 * self.raw_filled].clone()
            self.raw_base += drop
            self.raw_filled = keep
        self._h2d(self.raw[2 * self.raw_filled: 2 * (self.raw_filled + n)], x.reshape(-1))
        self.raw_filled += n
        self.n_in += n
        # outputs m whose last input floor((m*down + hl)/up) has arrived
        last = self.n_in * self.up - 1 - self.hl
        m_ready = last // self.down + 1 if last >= 0 else 0
        count = m_ready - self.m_next
        if count <= 0:
            return
        self._reserve_mono(count)
        self.eng.resample_range(self.raw.data_ptr(), self.raw_base, self.raw_filled, 2, self.stream_sr, self.sr,
                                self.m_next, count, self.mono.data_ptr() + 4 * self.filled, s)
        self.filled += count
        self.m_next = m_ready

    def push(self, stereo: np.ndarray) -> list[WindowResult]:
        """stereo: [n, 2] float32 host chunk at stream_sr. Returns the windows this chunk completed."""
        import torch

        x = np.ascontiguousarray(stereo, dtype=np.float32).reshape(-1, 2)
        s = torch.cuda.current_stream().cuda_stream
        if self.resampling:
            self._push_resampled(x, s)
        else:
            self._push_same_rate(x, s)
        starts = []
        while self.next_start + self.win <= self.base + self.filled:
            starts.append(self.next_start)
            self.next_start += self.hop
        if not starts:
            return []
        k = len(starts)
        offs = np.arange(k + 1, dtype=np.int64) * self.win
        if k == 1:  # one window (a push of <= one hop): extract it in place (even start: 8-B aligned)
            self.eng.extract_device(self.mono.data_ptr() + 4 * (starts[0] - self.base), offs, s)
        else:  # overlapping windows -> one contiguous clip each (device copies), one batched call
            if self.win_buf.numel() < k * self.win:
                self.win_buf = torch.empty(k * self.win, dtype=torch.float32, device="cuda")
            for i, st in enumerate(starts):
                r = st - self.base
                self.win_buf[i * self.win:(i + 1) * self.win] = self.mono[r:r + self.win]
            self.eng.extract_device(self.win_buf.data_ptr(), offs, s)
        rows = self.eng.query_extracted()
        return [WindowResult(st / self.sr, r) for st, r in zip(starts, rows)]

    def mono_history(self) -> np.ndarray:
        """Host copy of the mono buffer (index rate) currently held, from stream sample self.base."""
        return self.mono[: self.filled].cpu().numpy()


class StreamBank:
    """S live streams identified in lockstep (BASELINE config 5 at serving scale).

    Every push hands over the same length of interleaved stereo for every stream ([S, n, 2] float32, a device
    tensor or a host array). Per push the whole bank costs ONE K6 launch (aid_resample_batch_split: downmix + polyphase
    resampling of all S streams, reading the chunk where it lies and each stream's last few frames of the previous
    chunk from a small history, so chunked output equals whole-signal resampling bit for bit) and ONE extraction +
    match call over every window the push completed in every stream (aid_query_windows: K1-K3 read the 50 %-overlap
    windows in place from the streams' mono buffers, then K5).
    The reference's equivalent is one ffmpeg process and one `olaf_c query` per recorded clip
    (audio-ident-ui AudioRecorder.svelte:86-106 -> app/audio/decode.py:41-60 -> app/audio/fingerprint.py:158-219).
    """

    def __init__(self, engine, n_streams: int, stream_sr: int = 48000, window_s: float = 5.0, hop_s: float = 2.5,
                 capacity_s: float = 30.0):
        import torch

        self.eng = engine
        self.S = int(n_streams)
        self.sr = engine.sample_rate
        self.stream_sr = int(stream_sr)
        if self.stream_sr == self.sr:
            raise ValueError("StreamBank resamples: the stream rate must differ from the index rate "
                             "(StreamIdentifier handles same-rate streams)")
        self.win = int(round(window_s * self.sr)) & ~1
        self.hop = int(round(hop_s * self.sr)) & ~1
        self.up, self.down, self.hl, self.J = engine.resample_plan(self.stream_sr, self.sr)
        self.cap_m = max(int(capacity_s * self.sr), 4 * self.win) & ~1
        # K6 history: the input frames the next output still reads that came before the next chunk -- at most J - 1
        # per stream (the next output's last input has not arrived). Two buffers: the next history is written while
        # the launch that reads the current one may still be queued.
        self.hcap = (self.J + 1) & ~1
        self._hist = [torch.zeros(self.S, 2 * self.hcap, dtype=torch.float32, device="cuda") for _ in range(2)]
        self.hist_n = 0      # frames held per stream, ending at stream frame n_in
        self.mono = torch.zeros(self.S, self.cap_m, dtype=torch.float32, device="cuda")
        self._pin = None
        self._cur = None     # device copy of a host chunk
        self.n_in = 0        # frames received per stream
        self.m_next = 0      # next mono sample (index rate) to produce
        self.base = 0        # stream sample (index rate) of mono[:, 0]
        self.filled = 0
        self.next_start = 0  # stream sample of the next window
        self.timings = None  # a list: push() appends (append, resample, windows) host seconds per push (bench)

    def _chunk_dev(self, chunk, n: int):
        """The chunk on the device as [S, n, 2] with (frame, channel) contiguous per stream: (tensor, stream stride in
        floats). A device chunk is used in place (a strided slice of a longer stream tensor included)."""
        import torch

        if isinstance(chunk, torch.Tensor):
            t = chunk if chunk.dtype == torch.float32 else chunk.float()
            if not t.is_cuda:
                t = t.cuda()
            if n > 1 and (t.stride(2) != 1 or t.stride(1) != 2 or t.stride(0) % 2 or t.data_ptr() % 8):
                t = t.contiguous()
            return t, (t.stride(0) if self.S > 1 else 2 * n)
        x = np.ascontiguousarray(chunk, dtype=np.float32).reshape(self.S, 2 * n)
        if self._pin is None or self._pin.numel() < x.size:
            self._pin = torch.empty(x.size, dtype=torch.float32).pin_memory()
        if self._cur is None or self._cur.numel() < x.size:
            self._cur = torch.empty(x.size, dtype=torch.float32, device="cuda")
        torch.cuda.current_stream().synchronize()  # the previous chunk has left the staging buffer
        pin = self._pin[: x.size].view(self.S, 2 * n)
        pin.numpy()[:] = x
        cur = self._cur[: x.size].view(self.S, 2 * n)
        cur.copy_(pin, non_blocking=True)
        return cur.view(self.S, n, 2), 2 * n

    def _keep_history(self, cur, n: int) -> None:
        """The next history: stream frames [need, n_in) from the current history and the chunk (a few frames)."""
        need = max(0, (self.m_next * self.down + self.hl) // self.up - (self.J - 1))
        keep = self.n_in - need
        if keep > self.hcap:  # cannot happen: the next output's last input is >= n_in
            raise AssertionError("K6 history larger than J - 1 frames")
        old, new = self._hist
        from_cur = min(keep, n)
        from_old = keep - from_cur
        if from_old:
            new[:, : 2 * from_old] = old[:, 2 * (self.hist_n - from_old): 2 * self.hist_n]
        if from_cur:
            new[:, 2 * from_old: 2 * keep] = cur[:, n - from_cur: n].reshape(self.S, 2 * from_cur)
        self._hist = [new, old]
        self.hist_n = keep

    def push(self, chunk) -> list[list[WindowResult]]:
        """chunk: [S, n, 2] float32 at stream_sr (device tensor or host array). Returns, per stream, the windows this
        push completed (the same start times in every stream)."""
        return self._push(chunk, False)

    def push_submit(self, chunk) -> "PendingPush":
        """push() in two halves: the chunk's append and K6, then the extraction and match of the windows it completed
        are QUEUED (aid_query_windows_submit) and a PendingPush is returned at once; its collect() gives push()'s result.
        A serving loop submits push N + 1 before it collects push N, so the host work of one overlaps the kernels of
        the other."""
        return self._push(chunk, True)

    def _push(self, chunk, submit: bool):
        import torch

        n = int(chunk.shape[1])
        if chunk.shape[0] != self.S or (len(chunk.shape) > 2 and chunk.shape[2] != 2):
            raise ValueError("chunk must be [n_streams, n, 2]")
        s = torch.cuda.current_stream().cuda_stream
        t0 = time.perf_counter()
        cur, cur_stride = self._chunk_dev(chunk, n) if n else (None, 0)
        in_base = self.n_in
        self.n_in += n
        t1 = time.perf_counter()
        last = self.n_in * self.up - 1 - self.hl  # outputs m whose last input floor((m*down + hl)/up) has arrived
        m_ready = last // self.down + 1 if last >= 0 else 0
        count = m_ready - self.m_next
        if count > 0:
            if self.filled + count > self.cap_m:  # compact: keep what pending windows still need
                drop = (self.next_start - self.base) & ~1
                keep = self.filled - drop
                if keep + count > self.cap_m:
                    raise ValueError("chunk larger than the stream buffer")
                src = self.mono[:, drop: self.filled]
                self.mono[:, :keep] = src if keep <= drop else src.clone()
                self.base += drop
                self.filled = keep
            self.eng.resample_batch_split(self._hist[0].data_ptr(), 2 * self.hcap, self.hist_n,
                                          cur.data_ptr() if n else self._hist[0].data_ptr(), cur_stride, self.S,
                                          in_base, n, 2, self.stream_sr, self.sr, self.m_next, count,
                                          self.mono.data_ptr() + 4 * self.filled, self.cap_m, s)
            self.filled += count
            self.m_next = m_ready
        if n:
            self._keep_history(cur, n)
        t2 = time.perf_counter()
        starts = []
        while self.next_start + self.win <= self.base + self.filled:
            starts.append(self.next_start)
            self.next_start += self.hop
        if not starts:
            if self.timings is not None:
                self.timings.append((t1 - t0, t2 - t1, 0.0))
            return PendingPush(None, [], self.S, self.sr) if submit else [[] for _ in range(self.S)]
        rel = np.array(starts, dtype=np.int64) - self.base
        ws = (np.arange(self.S, dtype=np.int64)[:, None] * self.cap_m + rel[None, :]).ravel()
        if submit:
            pend = self.eng.query_windows_submit(self.mono.data_ptr(), ws, ws + self.win, s)
            if self.timings is not None:
                self.timings.append((t1 - t0, t2 - t1, time.perf_counter() - t2))
            return PendingPush(pend, starts, self.S, self.sr)
        rows = self.eng.query_windows(self.mono.data_ptr(), ws, ws + self.win, s)
        if self.timings is not None:
            self.timings.append((t1 - t0, t2 - t1, time.perf_counter() - t2))
        k = len(starts)
        return [[WindowResult(st / self.sr, rows[i * k + j]) for j, st in enumerate(starts)] for i in range(self.S)]


class PendingPush:
    """The windows of one StreamBank.push_submit, in flight on the GPU; collect() returns push()'s result."""

    __slots__ = ("pend", "starts", "S", "sr")

    def __init__(self, pend, starts, S: int, sr: int):
        self.pend, self.starts, self.S, self.sr = pend, starts, S, sr

    def collect(self) -> list[list[WindowResult]]:
        if self.pend is None:
            return [[] for _ in range(self.S)]
        rows = self.pend.collect()
        k = len(self.starts)
        return [[WindowResult(st / self.sr, rows[i * k + j]) for j, st in enumerate(self.starts)] for i in range(self.S)]
