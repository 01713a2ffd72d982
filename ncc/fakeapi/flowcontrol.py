"""A kube-apiserver's request admission, reduced to what a client sees: max-in-flight, API Priority and
Fairness seats with a bounded queue, and a per-write service time.

A real shard apiserver does not serve every request the moment it arrives.  Its filter chain caps the
mutating requests it holds (`--max-mutating-requests-inflight`, 200 by default) and, with API Priority and
Fairness (APF, on by default since 1.20), gives each priority level a number of *seats*: a request executes
on a free seat, waits in one of the level's bounded queues when none is free, and is answered
`429 Too Many Requests` with `Retry-After: 1` when its queue is full or its wait runs out.  Behind the seats
sits etcd, whose commit latency holds every write's seat for a while.  The controller's client
(native/executor/http.hpp `Client`, client-go's `rest` client in the reference — /root/reference/main.go:52-68)
has to live with that.  The fake apiserver's default serves every request at once on one core; with these
knobs set (`POST /_fake/faults`) it behaves like such a server:

  max_mutating_inflight   mutating requests admitted (queued or executing) at once; beyond → 429
  apf_seats               requests executing at once (one flow, one priority level); 0 = no APF model
  apf_queue               requests waiting for a seat; a full queue → 429
  apf_queue_wait_s        the longest a request waits for a seat before it is rejected (429)
  service_ms / read_service_ms   seat holding time per mutating / read request (etcd's commit latency)

Watches are long-running requests and, as on a real apiserver, exempt.  `stats()` counts what was
admitted, queued and rejected, and per wall-clock second how many requests arrived and how many were
rejected (bench/suite.py computes the 429 share after the first second of a cold start from it).
"""
from __future__ import annotations

import asyncio
import time
from collections import deque

from ..kube import errors as E


class FlowControl:
    def __init__(self):
        self.executing = 0
        self.mutating = 0  # admitted mutating requests, queued or executing
        self._queue: deque = deque()  # futures of requests waiting for a seat, FIFO
        self.counters = {"admitted": 0, "queued": 0, "rejected": 0, "rejected_inflight": 0,
                         "rejected_queue_full": 0, "rejected_queue_wait": 0, "max_executing": 0,
                         "max_queued": 0, "max_mutating": 0, "wait_max_s": 0.0}
        self.by_second: dict[int, list] = {}  # int(time.time()) -> [requests, rejected]

    @staticmethod
    def active(f) -> bool:
        return bool(f.apf_seats or f.max_mutating_inflight or f.service_ms or f.read_service_ms)

    def _reject(self, why: str) -> E.ApiError:
        self.counters["rejected"] += 1
        self.counters["rejected_" + why] += 1
        self.by_second[self._sec][1] += 1
        return E.TooManyRequests("too many requests, please try again later", retry_after=1)

    async def admit(self, f, mutating: bool) -> E.ApiError | None:
        """Hold a seat for one request (None), or the 429 to answer it with."""
        sec = self._sec = int(time.time())
        slot = self.by_second.get(sec)
        if slot is None:
            slot = self.by_second[sec] = [0, 0]
            if len(self.by_second) > 3600:
                for k in sorted(self.by_second)[:1800]:
                    del self.by_second[k]
        slot[0] += 1
        c = self.counters
        if mutating and f.max_mutating_inflight and self.mutating >= f.max_mutating_inflight:
            return self._reject("inflight")
        if f.apf_seats and (self.executing >= f.apf_seats or self._queue):
            if len(self._queue) >= max(0, int(f.apf_queue)):
                return self._reject("queue_full")
            fut = asyncio.get_running_loop().create_future()
            self._queue.append(fut)
            c["queued"] += 1
            c["max_queued"] = max(c["max_queued"], len(self._queue))
            if mutating:
                self.mutating += 1
            t0 = time.monotonic()
            try:
                await asyncio.wait_for(asyncio.shield(fut), f.apf_queue_wait_s)
            except asyncio.TimeoutError:
                if fut.done() and not fut.cancelled():  # the seat came as the wait ran out: give it back
                    self._seat_freed()
                else:
                    fut.cancel()
                if mutating:
                    self.mutating -= 1
                self._sec = int(time.time())
                self.by_second.setdefault(self._sec, [0, 0])
                return self._reject("queue_wait")
            c["wait_max_s"] = max(c["wait_max_s"], round(time.monotonic() - t0, 4))
            # the releasing request handed its seat over (`executing` already counts it)
        else:
            self.executing += 1
            if mutating:
                self.mutating += 1
        c["admitted"] += 1
        c["max_executing"] = max(c["max_executing"], self.executing)
        c["max_mutating"] = max(c["max_mutating"], self.mutating)
        return None

    def release(self, mutating: bool) -> None:
        if mutating:
            self.mutating -= 1
        self._seat_freed()

    def _seat_freed(self) -> None:
        while self._queue:
            fut = self._queue.popleft()
            if not fut.done():
                fut.set_result(None)  # the seat passes to the longest waiter
                return
        self.executing -= 1

    async def hold(self, f, mutating: bool) -> None:
        """The seat holding time of an admitted request (etcd's commit latency stand-in)."""
        ms = f.service_ms if mutating else f.read_service_ms
        if ms > 0:
            await asyncio.sleep(ms / 1000.0)

    def stats(self) -> dict:
        return dict(self.counters, executing=self.executing, waiting=len(self._queue), mutating=self.mutating,
                    by_second=[[s, v[0], v[1]] for s, v in sorted(self.by_second.items())])
