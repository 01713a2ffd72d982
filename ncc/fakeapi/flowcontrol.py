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

The model is callback-driven (no task or coroutine per request: `FakeApiServer.fast` hands the HTTP layer a
`Deferred` answered from a timer), so the substrate's own CPU does not become the bound the benchmark
compares the client against.
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
        self._queue: deque = deque()  # [granted callback, mutating, t_enqueued, live] of requests waiting for a seat
        self.counters = {"admitted": 0, "queued": 0, "rejected": 0, "rejected_inflight": 0,
                         "rejected_queue_full": 0, "rejected_queue_wait": 0, "max_executing": 0,
                         "max_queued": 0, "max_mutating": 0, "wait_max_s": 0.0}
        self.by_second: dict[int, list] = {}  # int(time.time()) -> [requests, rejected]

    @staticmethod
    def active(f) -> bool:
        return bool(f.apf_seats or f.max_mutating_inflight or f.service_ms or f.read_service_ms)

    def _slot(self) -> list:
        sec = int(time.time())
        slot = self.by_second.get(sec)
        if slot is None:
            slot = self.by_second[sec] = [0, 0]
            if len(self.by_second) > 3600:
                for k in sorted(self.by_second)[:1800]:
                    del self.by_second[k]
        return slot

    def _reject(self, why: str) -> E.ApiError:
        self.counters["rejected"] += 1
        self.counters["rejected_" + why] += 1
        self._slot()[1] += 1
        return E.TooManyRequests("too many requests, please try again later", retry_after=1)

    def _granted(self, mutating: bool, queued: bool) -> None:
        c = self.counters
        c["admitted"] += 1
        c["max_executing"] = max(c["max_executing"], self.executing)
        c["max_mutating"] = max(c["max_mutating"], self.mutating)

    def admit(self, f, mutating: bool, granted) -> E.ApiError | None:
        """Admit one request: the 429 to answer it with, or None — then `granted()` is called once it holds a
        seat (at once, or when one frees up)."""
        self._slot()[0] += 1
        if mutating and f.max_mutating_inflight and self.mutating >= f.max_mutating_inflight:
            return self._reject("inflight")
        if f.apf_seats and (self.executing >= f.apf_seats or self._queue):
            if len(self._queue) >= max(0, int(f.apf_queue)):
                return self._reject("queue_full")
            entry = [granted, mutating, time.monotonic(), True]
            self._queue.append(entry)
            c = self.counters
            c["queued"] += 1
            c["max_queued"] = max(c["max_queued"], len(self._queue))
            if mutating:
                self.mutating += 1
            asyncio.get_running_loop().call_later(f.apf_queue_wait_s, self._expire, entry)
            return None
        self.executing += 1
        if mutating:
            self.mutating += 1
        self._granted(mutating, False)
        granted()
        return None

    def _expire(self, entry: list) -> None:
        """A queued request's wait ran out: take it out of the queue and answer 429."""
        if not entry[3]:
            return  # it got its seat
        entry[3] = False
        try:
            self._queue.remove(entry)
        except ValueError:
            pass
        if entry[1]:
            self.mutating -= 1
        entry[0](self._reject("queue_wait"))

    def release(self, mutating: bool) -> None:
        """An admitted request finished: its seat passes to the longest waiter."""
        if mutating:
            self.mutating -= 1
        while self._queue:
            entry = self._queue.popleft()
            if not entry[3]:
                continue
            entry[3] = False
            c = self.counters
            c["wait_max_s"] = max(c["wait_max_s"], round(time.monotonic() - entry[2], 4))
            self._granted(entry[1], True)
            entry[0]()
            return
        self.executing -= 1

    @staticmethod
    def service_s(f, mutating: bool) -> float:
        """The seat holding time of an admitted request (etcd's commit latency stand-in)."""
        return (f.service_ms if mutating else f.read_service_ms) / 1000.0

    def stats(self) -> dict:
        return dict(self.counters, executing=self.executing, waiting=len(self._queue), mutating=self.mutating,
                    by_second=[[s, v[0], v[1]] for s, v in sorted(self.by_second.items())])
