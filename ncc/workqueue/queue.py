"""asyncio facade over a rate-limited work-queue core (native C++ by default, Python fallback).

`await queue.get()` parks the calling worker task until a key is ready, a delayed key
matures, or the queue shuts down — the asyncio equivalent of client-go's blocking
`workQueue.Get()` (controller.go:374).  Waiters are woken one per newly-available key, so a
burst of adds does not stampede every idle worker.

Also keeps the client-go workqueue metrics: adds, retries, depth, queue latency (time from
enqueue to hand-out) and work duration.
"""
from __future__ import annotations

import asyncio
import os
import time
from collections import deque

from .core import PyRateLimitingQueue

_FORCE_PY = os.environ.get("NCC_PURE_PYTHON_QUEUE", "") == "1"


def make_core(base_delay: float, max_delay: float, qps: float, burst: int, native: bool | None = None):
    """Build the queue core: `ncc._native.RateLimitingQueue` when available (or required)."""
    want_native = (not _FORCE_PY) if native is None else native
    if want_native:
        from .. import native as _n
        mod = _n.load(required=native is True)
        if mod is not None:
            return mod.RateLimitingQueue(float(base_delay), float(max_delay), float(qps), int(burst))
    return PyRateLimitingQueue(base_delay, max_delay, qps, burst)


class WorkQueue:
    def __init__(self, core=None, *, base_delay: float = 0.03, max_delay: float = 5.0, qps: float = 50.0,
                 burst: int = 300, native: bool | None = None, name: str = "controller"):
        self.core = core if core is not None else make_core(base_delay, max_delay, qps, burst, native)
        self.name = name
        self._waiters: deque[asyncio.Future] = deque()
        self._enqueued_at: dict[str, float] = {}
        self._timer: asyncio.TimerHandle | None = None
        self.metrics = {"adds": 0, "retries": 0, "gets": 0, "queue_latency_sum": 0.0, "work_sum": 0.0,
                        "max_depth": 0}
        self._started: dict[str, float] = {}

    @property
    def is_native(self) -> bool:
        return not isinstance(self.core, PyRateLimitingQueue)

    # ---------------------------------------------------------------- wakeups
    def _wake(self, n: int = 1) -> None:
        while n > 0 and self._waiters:
            f = self._waiters.popleft()
            if not f.done():
                f.set_result(None)
                n -= 1

    def _wake_all(self) -> None:
        self._wake(len(self._waiters))

    def _arm_timer(self) -> None:
        """Schedule a promotion at the earliest delayed key's ready time."""
        loop = asyncio.get_event_loop()
        now = time.monotonic()
        d = self.core.next_ready_in(now)
        if d < 0:
            return
        when = loop.time() + d
        if self._timer is not None and not self._timer.cancelled() and self._timer.when() <= when:
            return
        if self._timer is not None:
            self._timer.cancel()
        self._timer = loop.call_at(when, self._on_timer)

    def _on_timer(self) -> None:
        self._timer = None
        n = self.core.promote(time.monotonic())
        if n:
            self._wake(n)
        self._arm_timer()

    def _mark(self, key: str) -> None:
        if key not in self._enqueued_at:
            self._enqueued_at[key] = time.monotonic()

    # ---------------------------------------------------------------- API
    def add(self, key: str) -> None:
        self.metrics["adds"] += 1
        if self.core.add(key):
            self._mark(key)
            self._wake(1)
            depth = self.core.length()
            if depth > self.metrics["max_depth"]:
                self.metrics["max_depth"] = depth

    def add_after(self, key: str, delay: float) -> None:
        if self.core.add_after(key, float(delay), time.monotonic()):
            self._mark(key)
            self._wake(1)
        else:
            self._arm_timer()

    def add_rate_limited(self, key: str) -> float:
        self.metrics["retries"] += 1
        d = self.core.add_rate_limited(key, time.monotonic())
        if d <= 0 and self.core.length():
            self._mark(key)
            self._wake(1)
        self._arm_timer()
        return d

    def forget(self, key: str) -> None:
        self.core.forget(key)

    def num_requeues(self, key: str) -> int:
        return self.core.num_requeues(key)

    def done(self, key: str) -> None:
        t0 = self._started.pop(key, None)
        if t0 is not None:
            self.metrics["work_sum"] += time.monotonic() - t0
        if self.core.done(key):
            self._mark(key)
            self._wake(1)

    def busy(self, key: str) -> bool:
        return self.core.busy(key)

    def __len__(self) -> int:
        return self.core.length()

    def idle(self) -> bool:
        """Nothing queued and nothing being processed (delayed retries may still be pending)."""
        return self.core.length() == 0 and not self._started

    def shutdown(self) -> None:
        self.core.shutdown()
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        self._wake_all()

    def shutting_down(self) -> bool:
        return self.core.shutting_down()

    def try_get(self):
        key = self.core.try_get()
        if key is not None:
            self._handed_out(key)
        return key

    def _handed_out(self, key: str) -> None:
        now = time.monotonic()
        t = self._enqueued_at.pop(key, None)
        if t is not None:
            self.metrics["queue_latency_sum"] += now - t
        self.metrics["gets"] += 1
        self._started[key] = now

    async def get(self):
        """Next key, or None once the queue is shut down and drained of ready keys."""
        loop = asyncio.get_event_loop()
        while True:
            n = self.core.promote(time.monotonic())
            if n > 1:
                self._wake(n - 1)  # this caller takes one of the promoted keys; wake one waiter per other
            key = self.core.try_get()
            if key is not None:
                self._handed_out(key)
                return key
            if self.core.shutting_down():
                return None
            fut = loop.create_future()
            self._waiters.append(fut)
            self._arm_timer()
            try:
                await fut
            except asyncio.CancelledError:
                if not fut.done():
                    fut.cancel()
                raise
