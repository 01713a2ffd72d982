"""Pure-Python reference implementation of the rate-limited exclusive-key work queue.

Semantics are those of client-go `workqueue.NewTypedRateLimitingQueue` with
`NewTypedMaxOfRateLimiter(ItemExponentialFailure(base, max), Bucket(qps, burst))`
(controller.go:257-260,280):

* **dedup** — a key that is already waiting is not queued twice (`dirty` set);
* **exclusivity** — a key being processed is never handed to a second worker; re-adds while
  processing are parked and re-queued on `done` (`processing` set);
* **delays** — `add_after` parks a key in a min-heap until ready; an earlier ready time for an
  already-waiting key wins;
* **rate limiting** — only `add_rate_limited` consults the limiter; plain `add` bypasses it
  (SURVEY.md X9).  `forget` resets per-key backoff.

Time is passed in explicitly (`now`, seconds on the monotonic clock) so that this class and
the C++ `ncc._native.RateLimitingQueue` can be driven in lock-step by property tests.
The asyncio facade lives in `ncc.workqueue.queue`.
"""
from __future__ import annotations

import heapq
from collections import deque


class ItemExponentialFailureRateLimiter:
    def __init__(self, base_delay: float, max_delay: float):
        self.base, self.max = base_delay, max_delay
        self.failures: dict[str, int] = {}

    def when(self, key: str, now: float) -> float:
        exp = self.failures.get(key, 0)
        self.failures[key] = exp + 1
        if exp >= 64:
            return self.max
        d = self.base * (2.0 ** exp)
        return self.max if d > self.max else d

    def num_requeues(self, key: str) -> int:
        return self.failures.get(key, 0)

    def forget(self, key: str) -> None:
        self.failures.pop(key, None)


class BucketRateLimiter:
    """golang.org/x/time/rate reservation: tokens refill at qps up to burst, may go negative."""

    def __init__(self, qps: float, burst: int):
        self.qps, self.burst = float(qps), int(burst)
        self.tokens = float(burst)
        self.last: float | None = None

    def when(self, key: str, now: float) -> float:
        if self.qps <= 0:
            return 0.0
        if self.last is None:
            self.last = now
        elapsed = now - self.last
        if elapsed > 0:
            self.tokens = min(float(self.burst), self.tokens + elapsed * self.qps)
            self.last = now
        self.tokens -= 1.0
        return 0.0 if self.tokens >= 0 else -self.tokens / self.qps

    def num_requeues(self, key: str) -> int:
        return 0

    def forget(self, key: str) -> None:
        return None


class MaxOfRateLimiter:
    def __init__(self, *limiters):
        self.limiters = limiters

    def when(self, key: str, now: float) -> float:
        return max(l.when(key, now) for l in self.limiters)

    def num_requeues(self, key: str) -> int:
        return max(l.num_requeues(key) for l in self.limiters)

    def forget(self, key: str) -> None:
        for l in self.limiters:
            l.forget(key)


def default_controller_rate_limiter(base_delay: float, max_delay: float, qps: float, burst: int) -> MaxOfRateLimiter:
    return MaxOfRateLimiter(ItemExponentialFailureRateLimiter(base_delay, max_delay), BucketRateLimiter(qps, burst))


class PyRateLimitingQueue:
    """Same API as the native core (see module docstring)."""

    def __init__(self, base_delay: float = 0.005, max_delay: float = 1000.0, qps: float = 10.0, burst: int = 100,
                 limiter=None):
        self.limiter = limiter or default_controller_rate_limiter(base_delay, max_delay, qps, burst)
        self._queue: deque[str] = deque()
        self._dirty: set[str] = set()
        self._processing: set[str] = set()
        self._waiting: list[tuple[float, int, str]] = []  # (ready_at, seq, key)
        self._waiting_ready: dict[str, float] = {}
        self._seq = 0
        self._shutting_down = False

    # -- Type -----------------------------------------------------------------
    def add(self, key: str) -> bool:
        """Returns True when the key became available to `try_get` (caller wakes a worker)."""
        if self._shutting_down or key in self._dirty:
            return False
        self._dirty.add(key)
        if key in self._processing:
            return False
        self._queue.append(key)
        return True

    def try_get(self):
        if not self._queue:
            return None
        key = self._queue.popleft()
        self._processing.add(key)
        self._dirty.discard(key)
        return key

    def done(self, key: str) -> bool:
        self._processing.discard(key)
        if key in self._dirty:
            self._queue.append(key)
            return True
        return False

    def __len__(self) -> int:
        return len(self._queue)

    def length(self) -> int:
        return len(self._queue)

    def shutdown(self) -> None:
        self._shutting_down = True

    def shutting_down(self) -> bool:
        return self._shutting_down

    def processing(self) -> int:
        return len(self._processing)

    # -- Delaying ---------------------------------------------------------------
    def add_after(self, key: str, delay: float, now: float) -> bool:
        if self._shutting_down:
            return False
        if delay <= 0:
            return self.add(key)
        ready = now + delay
        prev = self._waiting_ready.get(key)
        if prev is not None and prev <= ready:
            return False
        self._waiting_ready[key] = ready
        self._seq += 1
        heapq.heappush(self._waiting, (ready, self._seq, key))
        return False

    def promote(self, now: float) -> int:
        """Move every waiting key whose ready time has passed into the queue."""
        n = 0
        w = self._waiting
        while w and w[0][0] <= now:
            ready, _, key = heapq.heappop(w)
            if self._waiting_ready.get(key) != ready:
                continue  # superseded by an earlier ready time
            del self._waiting_ready[key]
            if self.add(key):
                n += 1
        return n

    def next_ready_in(self, now: float) -> float:
        """Seconds until the earliest waiting key is ready; -1 if nothing is waiting."""
        w = self._waiting
        while w and self._waiting_ready.get(w[0][2]) != w[0][0]:
            heapq.heappop(w)
        if not w:
            return -1.0
        return max(0.0, w[0][0] - now)

    def waiting(self) -> int:
        return len(self._waiting_ready)

    def busy(self, key: str) -> bool:
        """Queued, being processed or waiting for a delayed add: a worker pass for the key is pending or running."""
        return key in self._dirty or key in self._processing or key in self._waiting_ready

    # -- RateLimiting -----------------------------------------------------------
    def add_rate_limited(self, key: str, now: float) -> float:
        d = self.limiter.when(key, now)
        self.add_after(key, d, now)
        return d

    def forget(self, key: str) -> None:
        self.limiter.forget(key)

    def num_requeues(self, key: str) -> int:
        return self.limiter.num_requeues(key)
