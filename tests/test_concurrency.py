"""aidfp.concurrency: the reader/writer lock and the query coalescer (CPU, no engine)."""

import threading
import time

import pytest

from aidfp.concurrency import QueryCoalescer, RWLock


def test_rwlock_readers_share_writer_excludes():
    lk = RWLock()
    lk.acquire_read()
    lk.acquire_read()  # two readers at once
    got = []
    w = threading.Thread(target=lambda: (lk.acquire_write(), got.append("w"), lk.release_write()))
    w.start()
    time.sleep(0.05)
    assert got == []  # the writer waits for both readers
    r3 = []
    t3 = threading.Thread(target=lambda: (lk.acquire_read(), r3.append(1), lk.release_read()))
    t3.start()
    time.sleep(0.05)
    assert r3 == []  # writer preference: a new reader queues behind the waiting writer
    lk.release_read()
    lk.release_read()
    w.join(5)
    t3.join(5)
    assert got == ["w"] and r3 == [1]


def test_coalescer_batches_and_keeps_order():
    seen = []

    def run(batch):
        seen.append(list(batch))
        time.sleep(0.01)
        return [x * 10 for x in batch]

    c = QueryCoalescer(run, window_s=0.002, max_batch=16)
    futs = [c.submit(i) for i in range(40)]
    assert [f.result(5) for f in futs] == [i * 10 for i in range(40)]
    assert sum(len(b) for b in seen) == 40
    assert max(len(b) for b in seen) <= 16 and len(seen) < 40
    assert [x for b in seen for x in b] == list(range(40))  # FIFO
    c.close()


def test_coalescer_propagates_errors_to_the_batch_only():
    def run(batch):
        if "bad" in batch:
            raise ValueError("boom")
        return batch

    c = QueryCoalescer(run, window_s=0.0)
    assert c.submit("ok").result(5) == "ok"
    f = c.submit("bad")
    with pytest.raises(ValueError):
        f.result(5)
    assert c("fine") == "fine"  # the dispatcher survives
    c.close()


def test_coalescer_lone_request_latency():
    c = QueryCoalescer(lambda b: b, window_s=0.0005)
    c("warm")
    t = time.perf_counter()
    for _ in range(50):
        c("x")
    assert (time.perf_counter() - t) / 50 < 0.01
    c.close()


def test_coalescer_window_opens_only_under_load():
    """A lone request (the previous batch was one request) is dispatched at once, even with a long window; after a
    batch of several requests the window collects the next ones."""
    import threading

    seen = []
    gate = threading.Event()

    def run(batch):
        seen.append(len(batch))
        gate.wait(5)
        return batch

    c = QueryCoalescer(run, window_s=0.2, max_batch=64)
    gate.set()
    t = time.perf_counter()
    for _ in range(5):
        c("x")
    assert (time.perf_counter() - t) / 5 < 0.05  # no 0.2 s window per lone request
    gate.clear()
    first = c.submit("a")  # occupies the dispatcher
    time.sleep(0.05)
    futs = [c.submit(i) for i in range(8)]  # queue up behind it
    gate.set()
    first.result(5)
    assert [f.result(5) for f in futs] == list(range(8))
    assert seen[-1] == 8  # taken together
    c.close()


def test_coalescer_async_requests_resolved_per_batch():
    """submit_async (olaf_query's path): every coroutine gets its own result, in one thread-safe callback per loop
    and batch rather than one per request; a failing batch fails its requests only; a request cancelled while its
    batch runs is skipped."""
    import asyncio

    release = threading.Event()

    def run(batch):
        release.wait(5)
        if any(p == "bad" for p in batch):
            raise ValueError("bad batch")
        return [p * 2 for p in batch]

    c = QueryCoalescer(run, window_s=0.05)
    calls = []

    async def main():
        loop = asyncio.get_running_loop()
        orig = loop.call_soon_threadsafe

        def counting(cb, *a, **k):
            calls.append(cb)
            return orig(cb, *a, **k)

        loop.call_soon_threadsafe = counting
        first = c.submit_async(0)  # a lone first batch: dispatched at once
        await asyncio.sleep(0.01)
        futs = [c.submit_async(i) for i in range(1, 33)]  # queued while batch 1 waits: one batch of 32
        release.set()
        assert await first == 0
        res = await asyncio.gather(*futs)
        assert res == [2 * i for i in range(1, 33)]
        n_before = len(calls)
        bad = [c.submit_async("bad"), c.submit_async(5)]
        out = await asyncio.gather(*bad, return_exceptions=True)
        assert all(isinstance(x, ValueError) for x in out)
        assert len(calls) - n_before <= 2
        late = c.submit_async(7)
        late.cancel()
        assert await c.submit_async(8) == 16
        return len(calls)

    try:
        n = asyncio.run(main())
    finally:
        c.close()
    # batches: {0}, {1..32}, {bad, 5} (maybe split), {7, 8} (maybe split): far fewer callbacks than the 37 requests
    assert n <= 8, n


class _Handle:
    def __init__(self, log, batch, gate, fail=False):
        self.log, self.batch, self.gate, self.fail = log, batch, gate, fail

    def collect(self):
        self.gate.wait(5)
        self.log.append(("collect", list(self.batch)))
        if self.fail:
            raise ValueError("collect failed")
        return [x * 10 for x in self.batch]


def test_coalescer_pipelined_dispatch_overlaps_and_keeps_results():
    """submit_batch (the service's aid_query_pcm_submit path): under load the dispatcher starts batch N + 1 before it
    collects batch N; every request still gets its own result, FIFO, and a lone request is answered at once."""
    log = []
    gate = threading.Event()
    gate.set()

    def submit(batch, behind):
        log.append(("submit", list(batch), behind))
        return _Handle(log, batch, gate)

    c = QueryCoalescer(lambda b: pytest.fail("synchronous runner used"), window_s=0.002, max_batch=8,
                       submit_batch=submit)
    assert c(3) == 30  # lone request: submitted and collected at once (nothing to overlap with)
    gate.clear()
    futs = [c.submit(i) for i in range(40)]
    time.sleep(0.05)
    gate.set()
    assert [f.result(5) for f in futs] == [i * 10 for i in range(40)]
    subs = [e for e in log if e[0] == "submit"]
    assert [x for e in subs[1:] for x in e[1]] == list(range(40))  # FIFO
    assert c.overlapped > 0 and any(e[2] for e in subs)
    # the overlap: some batch is submitted before the previous one is collected
    order = [(e[0], tuple(e[1])) for e in log]
    assert any(order[i][0] == "submit" and order[i + 1][0] == "collect" and order[i][1] != order[i + 1][1]
               for i in range(len(order) - 1))
    c.close()


def test_coalescer_pipelined_busy_and_failures():
    """A runner that declines a batch beside the outstanding one (a writer waits for the index lock) is called again
    once that batch is collected; a failing submit or collect fails its own batch only."""
    log = []
    gate = threading.Event()
    gate.set()
    declined = []

    def submit(batch, behind):
        if "bad-submit" in batch:
            raise ValueError("submit failed")
        if behind and len(declined) < 3:
            declined.append(list(batch))
            return None
        log.append(("submit", list(batch), behind))
        return _Handle(log, batch, gate, fail="bad-collect" in batch)

    c = QueryCoalescer(lambda b: pytest.fail("synchronous runner used"), window_s=0.002, max_batch=4,
                       submit_batch=submit)
    gate.clear()
    futs = [c.submit(i) for i in range(20)]
    time.sleep(0.05)
    gate.set()
    assert [f.result(5) for f in futs] == [i * 10 for i in range(20)]
    assert len(declined) == 3  # each declined batch ran after the outstanding one, not lost
    for bad in ("bad-submit", "bad-collect"):
        f = c.submit(bad)
        with pytest.raises(ValueError):
            f.result(5)
        assert c(2) == 20  # the dispatcher survives
    c.close()


def test_rwlock_try_read():
    lk = RWLock()
    assert lk.try_acquire_read()
    w = threading.Thread(target=lambda: (lk.acquire_write(), lk.release_write()))
    w.start()
    time.sleep(0.05)
    assert not lk.try_acquire_read()  # a writer waits: no second hold without waiting
    lk.release_read()
    w.join(5)
    assert lk.try_acquire_read()
    lk.release_read()
