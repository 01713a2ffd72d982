"""Client-side token-bucket rate limiting (client-go flowcontrol / golang.org/x/time/rate semantics).

client-go gives every API-group REST client its own `NewTokenBucketRateLimiter(QPS, Burst)`,
defaulting to 5 QPS / burst 10 when `rest.Config.QPS == 0` — which is what the reference runs
with, since main.go:52-68 never sets QPS.  Reference-compat mode
reproduces that; native mode defaults to unlimited.
"""
from __future__ import annotations

import asyncio
import time


class TokenBucket:
    """rate.Limiter reservation arithmetic: tokens refill at `qps` up to `burst`; a reservation
    takes one token and may drive the balance negative, the deficit being the wait."""

    __slots__ = ("qps", "burst", "_tokens", "_last")

    def __init__(self, qps: float, burst: int, now: float | None = None):
        self.qps = float(qps)
        self.burst = max(int(burst), 1)
        self._tokens = float(self.burst)
        self._last = time.monotonic() if now is None else now

    def reserve(self, now: float) -> float:
        """Take one token at time `now`; return the delay (seconds) before it may be used."""
        if self.qps <= 0:
            return 0.0
        elapsed = max(0.0, now - self._last)
        self._tokens = min(float(self.burst), self._tokens + elapsed * self.qps)
        self._last = now
        self._tokens -= 1.0
        if self._tokens >= 0:
            return 0.0
        return -self._tokens / self.qps


class AsyncRateLimiter:
    """awaitable wrapper: `await limiter.wait()` blocks the caller for its reservation delay."""

    def __init__(self, qps: float, burst: int):
        self.bucket = TokenBucket(qps, burst)
        self.enabled = qps > 0
        self.waited_s = 0.0  # cumulative throttle time, exported as a metric

    async def wait(self) -> None:
        if not self.enabled:
            return
        d = self.bucket.reserve(time.monotonic())
        if d > 0:
            self.waited_s += d
            await asyncio.sleep(d)
