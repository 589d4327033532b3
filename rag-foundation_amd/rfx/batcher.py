"""Group-commit micro-batching of concurrent search requests.

The reference's chat route runs every request in its own thread (up to 50 per process,
chat.py:40,496-521) and each calls the retriever for ONE question.  On the GPU a query costs
nearly the same alone as inside a 256-query batch (the scan streams the whole index either way),
so concurrent questions should share one launch.

GroupBatcher: the first caller to find the batcher idle becomes the leader and runs a batch of
everything queued at that moment (up to max_batch); requests that arrive while a batch runs wait,
and when it finishes leadership passes to the oldest of them, which runs the next batch.  No
timer, no background thread (safe across gunicorn forks): an idle process adds no latency, a busy
one forms batches as large as the queue that built up during the previous launch.
"""
import os
import threading
from typing import Any, Callable, List, Sequence


class BatchTimeout(TimeoutError):
    """A waiter gave up: the batch ahead of it did not finish in time.  A TimeoutError, so the
    reference's retry paths apply (RETRYABLE_EXCEPTIONS, gemini_rag.py:17-27; chat retries before
    the first delta, chat.py:1076-1128)."""


class _Slot:
    __slots__ = ("event", "result", "error", "lead")

    def __init__(self):
        self.event = threading.Event()
        self.result = None
        self.error = None
        self.lead = False


class GroupBatcher:
    def __init__(self, run: Callable[[Sequence[Any]], List[Any]], max_batch: int = 256, timeout: float = None):
        """run(items) -> results, one per item, in order; called by one thread at a time.
        timeout: longest a request waits for the batches ahead of it (RFX_BATCH_TIMEOUT_S, 30 s)
        before it raises BatchTimeout; a request that is running its own batch is not cut off."""
        if max_batch < 1:
            raise ValueError("max_batch must be >= 1")
        self._run = run
        self.max_batch = int(max_batch)
        self.timeout = float(os.environ.get("RFX_BATCH_TIMEOUT_S", "30")) if timeout is None else float(timeout)
        self._lock = threading.Lock()
        self._queue: List[tuple] = []
        self._busy = False
        self.batches = 0  # statistics (tests / metrics)
        self.items = 0

    def submit(self, item: Any) -> Any:
        slot = _Slot()
        with self._lock:
            self._queue.append((item, slot))
            lead = not self._busy
            self._busy = True
        if not lead:
            if not slot.event.wait(self.timeout):
                with self._lock:
                    queued = any(s is slot for _, s in self._queue)
                    if queued and not slot.lead:
                        self._queue = [(it, s) for it, s in self._queue if s is not slot]
                        raise BatchTimeout(f"search queue: no batch slot within {self.timeout:.0f} s")
                # handed the lead at the deadline, or already inside a running batch
                if not slot.lead and not slot.event.wait(self.timeout):
                    raise BatchTimeout(f"search batch did not finish within {2 * self.timeout:.0f} s")
            if not slot.lead:
                return self._value(slot)
            slot.event.clear()
        self._run_one()
        slot.event.wait()
        return self._value(slot)

    @staticmethod
    def _value(slot: _Slot):
        if slot.error is not None:
            raise slot.error
        return slot.result

    def _run_one(self):
        with self._lock:
            batch = self._queue[: self.max_batch]
            del self._queue[: self.max_batch]
        try:
            results = self._run([it for it, _ in batch])
            if len(results) != len(batch):
                raise RuntimeError(f"batch runner returned {len(results)} results for {len(batch)} items")
            for (_, slot), res in zip(batch, results):
                slot.result = res
        except BaseException as e:  # every waiter of this batch sees the failure
            for _, slot in batch:
                slot.error = e
        finally:
            with self._lock:
                self.batches += 1
                self.items += len(batch)
                nxt = self._queue[0][1] if self._queue else None
                if nxt is None:
                    self._busy = False
                else:
                    nxt.lead = True  # hand over: the oldest waiter runs the next batch
            for _, slot in batch:
                slot.event.set()
            if nxt is not None:
                nxt.event.set()
