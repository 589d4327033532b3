"""CPU: group-commit micro-batching (rfx.batcher.GroupBatcher) — every caller gets its own result,
concurrent callers share batches, failures reach exactly the callers of the failed batch, and an
idle batcher adds no waiting (a lone caller runs a batch of one at once)."""
import threading
import time

import pytest

from rfx.batcher import GroupBatcher


def test_sequential_calls_run_batches_of_one():
    seen = []
    b = GroupBatcher(lambda items: (seen.append(list(items)), [x * 2 for x in items])[1])
    assert [b.submit(i) for i in range(5)] == [0, 2, 4, 6, 8]
    assert seen == [[0], [1], [2], [3], [4]]
    assert b.batches == 5 and b.items == 5


def test_concurrent_callers_share_batches_and_get_their_own_results():
    sizes = []

    def run(items):
        sizes.append(len(items))
        time.sleep(0.02)  # a "GPU launch": requests pile up meanwhile
        return [(x, x * x) for x in items]

    b = GroupBatcher(run, max_batch=16)
    out = {}
    start = threading.Barrier(64)

    def worker(i):
        start.wait()
        out[i] = b.submit(i)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(64)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
    assert all(out[i] == (i, i * i) for i in range(64))
    assert sum(sizes) == 64 and max(sizes) <= 16
    assert len(sizes) < 64  # batching happened
    assert b.items == 64


def test_failure_reaches_only_its_batch():
    calls = []

    def run(items):
        calls.append(list(items))
        if "bad" in items:
            raise ValueError("boom")
        return [x.upper() for x in items]

    b = GroupBatcher(run)
    with pytest.raises(ValueError):
        b.submit("bad")
    assert b.submit("ok") == "OK"  # the batcher recovered (not stuck busy)


def test_wrong_result_count_is_an_error():
    # force a 2-item batch: hold the runner while two callers queue
    gate = threading.Event()
    b2 = GroupBatcher(lambda items: (gate.wait(5), [0])[1])
    res = []
    t1 = threading.Thread(target=lambda: res.append(b2.submit(1)))
    t1.start()
    time.sleep(0.05)
    errs = []

    def later(v):
        try:
            res.append(b2.submit(v))
        except RuntimeError as e:
            errs.append(e)

    t2 = threading.Thread(target=later, args=(2,))
    t3 = threading.Thread(target=later, args=(3,))
    t2.start()
    t3.start()
    time.sleep(0.05)
    gate.set()
    for t in (t1, t2, t3):
        t.join(timeout=10)
    assert res[0] == 0 and len(errs) == 2  # the 2-item batch got 1 result: both callers fail


def test_many_rounds_no_deadlock():
    b = GroupBatcher(lambda items: list(items), max_batch=3)
    N = 200
    got = []
    lock = threading.Lock()

    def worker(i):
        for j in range(5):
            v = b.submit((i, j))
            with lock:
                got.append(v)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(N // 5)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=60)
    assert sorted(got) == sorted((i, j) for i in range(N // 5) for j in range(5))


def test_bad_max_batch():
    with pytest.raises(ValueError):
        GroupBatcher(lambda items: items, max_batch=0)


def test_waiter_times_out_with_a_retryable_error_and_leaves_the_queue():
    """A hung launch must not block every chat thread forever: a queued
    caller gives up after the batcher's timeout with a TimeoutError (retryable, gemini_rag.py:
    17-27) and is removed from the queue, so the next batch does not run its request."""
    from rfx.batcher import BatchTimeout

    release = threading.Event()
    ran = []

    def run(items):
        ran.append(list(items))
        if items[0] == "slow":
            release.wait(5)
        return list(items)

    b = GroupBatcher(run, timeout=0.2)
    t = threading.Thread(target=lambda: b.submit("slow"))
    t.start()
    time.sleep(0.05)
    t0 = time.monotonic()
    with pytest.raises(TimeoutError) as ei:
        b.submit("waiter")
    assert isinstance(ei.value, BatchTimeout) and time.monotonic() - t0 < 2
    release.set()
    t.join(timeout=5)
    assert b.submit("after") == "after"
    assert ["waiter"] not in ran and ran[-1] == ["after"]
