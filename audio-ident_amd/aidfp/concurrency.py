"""Concurrent readers at the boundary (SURVEY.md 8b "reentrant aid_query under shared lock").

The reference runs one `olaf_c query` subprocess per request
(audio-ident-service/app/audio/fingerprint.py:185-193), so concurrent searches query in
parallel, while LMDB keeps a single writer (fingerprint.py:7-8, routers/ingest.py:49-52).
Here the index lives in one GPU engine:

  * `RWLock` -- index writers (store, delete, checkpoint) are exclusive; readers share.
  * `QueryCoalescer` -- concurrent query requests are gathered into ONE engine call
    (aid_query_pcm: K1-K3 + K5 over the whole batch). A dispatcher thread takes the first
    waiting request, collects whatever else arrives within `window_s` (up to `max_batch`),
    runs the batch under the read lock and resolves every request's future. Under load the
    next batch accumulates while the current one runs on the GPU, so batching follows the
    arrival rate. The window only opens after a batch of more than one request: at low load
    (the previous batch was a lone request) a request is dispatched at once and pays no window.
    Requests from an asyncio event loop (`submit_async`, what `olaf_query` uses) are resolved
    with ONE thread-safe callback per loop and batch instead of one per request: at 64 clients
    the per-request wake-ups of `asyncio.wrap_future` were most of the service's host time.
"""

from __future__ import annotations

import asyncio
import collections
import logging
import queue
import threading
import time
from concurrent.futures import Future
from typing import Callable, Sequence

logger = logging.getLogger(__name__)


class RWLock:
    """Writer-preferring reader/writer lock (a waiting writer blocks new readers)."""

    def __init__(self):
        self._cv = threading.Condition(threading.Lock())
        self._readers = 0
        self._writer = False
        self._writers_waiting = 0

    def acquire_read(self) -> None:
        with self._cv:
            while self._writer or self._writers_waiting:
                self._cv.wait()
            self._readers += 1

    def try_acquire_read(self) -> bool:
        """A read hold only if it needs no wait (no writer holds or awaits the lock). A thread that already holds
        a read hold takes a second one with this: a blocking acquire behind a waiting writer would deadlock."""
        with self._cv:
            if self._writer or self._writers_waiting:
                return False
            self._readers += 1
            return True

    def release_read(self) -> None:
        with self._cv:
            self._readers -= 1
            if self._readers == 0:
                self._cv.notify_all()

    def acquire_write(self) -> None:
        with self._cv:
            self._writers_waiting += 1
            try:
                while self._writer or self._readers:
                    self._cv.wait()
            finally:
                self._writers_waiting -= 1
            self._writer = True

    def release_write(self) -> None:
        with self._cv:
            self._writer = False
            self._cv.notify_all()

    class _Guard:
        def __init__(self, acq, rel):
            self._acq, self._rel = acq, rel

        def __enter__(self):
            self._acq()
            return self

        def __exit__(self, *exc):
            self._rel()

    def read(self) -> "RWLock._Guard":
        return RWLock._Guard(self.acquire_read, self.release_read)

    def write(self) -> "RWLock._Guard":
        return RWLock._Guard(self.acquire_write, self.release_write)


_STOP = object()
_BUSY = object()  # QueryCoalescer._start: the runner declined to start a batch beside the outstanding one


class _LoopFuture:
    """An asyncio future of `loop`, resolved from the dispatcher thread through the loop (see _dispatch)."""

    __slots__ = ("loop", "fut")

    def __init__(self, loop, fut):
        self.loop, self.fut = loop, fut

    def set_running_or_notify_cancel(self) -> bool:
        return not self.fut.cancelled()  # a read from another thread: a late cancel is caught in _resolve


def _resolve(items) -> None:
    """In the event loop: [(asyncio future, result, exception)] of one batch."""
    for fut, res, exc in items:
        if fut.done():  # cancelled while its batch ran
            continue
        if exc is not None:
            fut.set_exception(exc)
        else:
            fut.set_result(res)


def _size(payload) -> int:
    """Bytes of a request payload for the batch cap (0 for payloads without a length)."""
    try:
        return len(payload)
    except TypeError:
        return 0


class QueryCoalescer:
    """Gathers concurrent requests into batches for `run_batch(payloads) -> results` (same order).

    A batch closes at `max_batch` requests or when the next request would take its payload bytes
    (`len(payload)`) past `max_batch_bytes` (that request opens the next batch; a single request larger
    than the cap runs alone), so many long uploads never land in one engine call."""

    def __init__(self, run_batch: Callable[[Sequence], Sequence], window_s: float = 0.0005, max_batch: int = 256,
                 max_batch_bytes: int = 64 << 20, workers: int = 1,
                 submit_batch: Callable[[Sequence, bool], object] | None = None, split_min: int = 0,
                 split_parts: int = 2):
        self._run = run_batch
        # pipelined dispatch: submit_batch(payloads, behind) starts a batch and returns a handle
        # whose collect() gives the results; the dispatcher starts batch N + 1 before it collects batch N, so one
        # batch's host work (gathering, the PCM copy into page-locked memory, row parsing, resolution) runs while
        # the other batch's copy and kernels do. `behind` says a batch is still outstanding: the runner may then
        # decline with None (e.g. a writer waits for the index lock) and is called again once that batch is done.
        self._submit = submit_batch
        # closed-loop clients answered together come back together: one batch in flight and nothing to overlap it
        # with. With split_min > 0, a pipelined batch of at least split_min requests gathered while none is
        # outstanding is started as two halves, so the first half's answers (and its clients' next requests) overlap
        # the second half's copy and kernels.
        self.split_min = int(split_min)
        self.split_parts = max(2, int(split_parts))  # parts of a split batch = batches in flight at most
        self.window_s = float(window_s)
        self.max_batch = int(max_batch)
        self.max_batch_bytes = int(max_batch_bytes)
        # dispatcher threads: with two, one batch's host work runs while the other batch is inside its engine call
        # (which releases the GIL); the engine itself still runs one call at a time. With submit_batch the single
        # dispatcher overlaps its batches itself.
        self.workers = max(1, int(workers))
        self._last_batch = 0  # size of the previous batch: the collection window opens only after a batch > 1
        self._q: queue.SimpleQueue = queue.SimpleQueue()
        self._threads: list[threading.Thread] = []
        self._start_lock = threading.Lock()
        self._batches_lock = threading.Lock()
        self.batches: list[int] = []  # sizes of the last batches run (bounded; tests and stats)
        self.overlapped = 0  # batches started while another was outstanding (pipelined dispatch)

    def submit(self, payload) -> Future:
        fut: Future = Future()
        self._ensure_thread()
        self._q.put((payload, fut))
        return fut

    def submit_async(self, payload) -> "asyncio.Future":
        """From a running event loop: an asyncio future of this request's result."""
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._ensure_thread()
        self._q.put((payload, _LoopFuture(loop, fut)))
        return fut

    def __call__(self, payload):
        return self.submit(payload).result()

    def close(self) -> None:
        with self._start_lock:
            ts, self._threads = self._threads, []
        for _ in ts:
            self._q.put(_STOP)
        for t in ts:
            t.join()

    def _ensure_thread(self) -> None:
        if self._threads:
            return
        with self._start_lock:
            if not self._threads:
                ts = [threading.Thread(target=self._loop, name=f"aidfp-query-coalescer-{i}", daemon=True)
                      for i in range(self.workers)]
                for t in ts:
                    t.start()
                self._threads = ts

    def _gather(self, first):
        """The batch that `first` opens: what is queued now or arrives within the window, up to the caps.
        Returns (batch, held request or None, stop seen)."""
        batch = [first]
        nbytes = _size(first[0])
        held = None
        # low load (the previous batch was one request): dispatch what is queued now, no wait for company
        window = self.window_s if self._last_batch > 1 else 0.0
        deadline = time.monotonic() + window
        while len(batch) < self.max_batch:
            try:
                item = self._q.get_nowait()
            except queue.Empty:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    item = self._q.get(timeout=left)
                except queue.Empty:
                    break
            if item is _STOP:
                return batch, held, True
            if nbytes + _size(item[0]) > self.max_batch_bytes:
                held = item  # opens the next batch
                break
            nbytes += _size(item[0])
            batch.append(item)
        return batch, held, False

    def _loop(self) -> None:
        pipelined = self._submit is not None and self.workers == 1
        depth = self.split_parts  # batches in flight at most (pipelined dispatch)
        held = None  # the request that did not fit this thread's previous batch
        inflight: collections.deque = collections.deque()  # (live requests, handle, exception), oldest first
        while True:
            if held is not None:
                first, held = held, None
            elif not inflight:
                first = self._q.get()
            else:
                try:
                    first = self._q.get_nowait()
                except queue.Empty:  # nothing to overlap the oldest batch in flight with: answer it now
                    self._finish(*inflight.popleft())
                    continue
            if first is _STOP:
                while inflight:
                    self._finish(*inflight.popleft())
                return
            batch, held, stop = self._gather(first)
            if pipelined:
                parts = [batch]
                if not inflight and self.split_min and len(batch) >= self.split_min:
                    k = min(depth, len(batch))
                    parts = [batch[i * len(batch) // k:(i + 1) * len(batch) // k] for i in range(k)]
                for part in parts:
                    live = self._live(part)
                    if not live:
                        continue
                    while len(inflight) >= depth:
                        self._finish(*inflight.popleft())
                    started = self._start(live, bool(inflight))
                    if started is _BUSY:  # the runner cannot start this batch beside the outstanding ones
                        while inflight:
                            self._finish(*inflight.popleft())
                        started = self._start(live, False)
                    elif inflight:
                        self.overlapped += 1
                    inflight.append(started)
                while len(inflight) > depth - 1:  # the newest stays in flight while the next batch gathers
                    self._finish(*inflight.popleft())
            else:
                self._dispatch(batch)
            if stop:
                while inflight:
                    self._finish(*inflight.popleft())
                if held is not None:
                    self._dispatch([held])
                return

    def _live(self, batch) -> list:
        self._last_batch = len(batch)
        with self._batches_lock:
            self.batches.append(len(batch))
            del self.batches[:-1024]
        return [(p, f) for p, f in batch if f.set_running_or_notify_cancel()]

    def _start(self, live, behind: bool):
        try:
            h = self._submit([p for p, _ in live], behind)
        except BaseException as exc:  # every request of the batch sees the failure
            return live, None, exc
        if h is None:
            if not behind:
                return live, None, RuntimeError("batch runner declined a batch with none outstanding")
            return _BUSY
        return live, h, None

    def _finish(self, live, handle, exc) -> None:
        if exc is None:
            try:
                results = handle.collect()
                if len(results) != len(live):
                    raise RuntimeError(f"batch runner returned {len(results)} results for {len(live)} requests")
            except BaseException as e:
                exc = e
        self._resolve_all(live, [(r, None) for r in results] if exc is None else [(None, exc)] * len(live))

    def _dispatch(self, batch) -> None:
        live = self._live(batch)
        if not live:
            return
        try:
            results = self._run([p for p, _ in live])
            if len(results) != len(live):
                raise RuntimeError(f"batch runner returned {len(results)} results for {len(live)} requests")
            outcome = [(r, None) for r in results]
        except BaseException as exc:  # every request of the batch sees the failure
            outcome = [(None, exc)] * len(live)
        self._resolve_all(live, outcome)

    @staticmethod
    def _resolve_all(live, outcome) -> None:
        per_loop: dict = {}
        for (_, f), (r, exc) in zip(live, outcome):
            if isinstance(f, _LoopFuture):
                per_loop.setdefault(f.loop, []).append((f.fut, r, exc))
            elif exc is not None:
                f.set_exception(exc)
            else:
                f.set_result(r)
        for loop, items in per_loop.items():
            try:
                loop.call_soon_threadsafe(_resolve, items)
            except RuntimeError:  # the loop was closed meanwhile: nobody awaits these any more
                pass
