"""Kubernetes Event recording: recorder → broadcaster → correlator → sink.

The reference builds `record.NewBroadcaster` with structured logging and a sink writing to
the controller cluster (controller.go:252-256); recorded reasons are in controller.go:60-81.
This module re-creates the parts of client-go `tools/record` that shape the API traffic:

* non-blocking `event()` into a bounded buffer (client-go drops on overflow, 1000 entries);
* the **spam filter**: a token bucket per (source, involved object), burst 25, refill 1/300 s;
* **aggregation**: >10 distinct messages for the same (object, type, reason) within 10 minutes
  collapse into one "(combined from similar events): …" event;
* **dedup**: a repeat of an identical event PATCHes `count`/`lastTimestamp` of the existing
  Event instead of creating a new one;
* bounded retries of failed sink writes.

The correlator runs when an event is recorded, as client-go's broadcaster does on receipt.  With
`coalesce=True` (native mode) an event identical to one still waiting for its writer is folded into it:
one write then carries both (`count` + n).  The Event object ends up the same — count, last
timestamp, message — with fewer API writes when a burst outruns the writers.  With `repeat_window` > 0
(native mode, `event-repeat-window`) a repeat of an event that has already been written is held for up to
that long and folded with the repeats that follow it: a template synced on every wave of a rollout costs one
count PATCH per window instead of one per pass (a first occurrence, and every Warning that is new, still goes
out at once).

`FakeRecorder` mirrors client-go's: it keeps "Type Reason Message" strings (or drops them).
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..aio import wait_timeout
from ..api import constants as C
from ..api import resources as R
from ..api.objects import meta, now_rfc3339
from ..kube.client import PATCH_STRATEGIC, KubeClient
from ..kube.ratelimit import TokenBucket

log = logging.getLogger("ncc.events")

SPAM_BURST = 25
SPAM_QPS = 1.0 / 300.0
AGGREGATE_MAX_EVENTS = 10
AGGREGATE_INTERVAL_S = 600.0
BUFFER = 1000
WARNING_OVERFLOW = 16384  # native: Warnings held past a full buffer (beyond this they are dropped too)


class EventRecorder:
    def event(self, obj: dict, event_type: str, reason: str, message: str, kind: str | None = None) -> None:
        raise NotImplementedError


CACHE_LIMIT = 4096  # client-go's maxLruCacheEntries


def _bound(cache: dict, limit=CACHE_LIMIT) -> None:
    """Keep a correlator cache within `limit` entries (client-go: 4096, maxLruCacheEntries): past the limit
    the oldest quarter goes (insertion order), so a controller that has seen many objects does not grow.
    `limit` may be a callable, evaluated only when the cache is over the default."""
    n = len(cache)
    if n <= CACHE_LIMIT:
        return
    if callable(limit):
        limit = max(CACHE_LIMIT, int(limit()))
    if n > limit:
        for k in list(cache)[:limit // 4]:
            del cache[k]


class FakeRecorder(EventRecorder):
    """client-go record.FakeRecorder: with `keep=False` events are discarded (as in the reference tests)."""

    def __init__(self, keep: bool = True):
        self.keep = keep
        self.events: list[str] = []

    def event(self, obj, event_type, reason, message, kind=None):
        if self.keep:
            self.events.append(f"{event_type} {reason} {message}")


def involved_object(obj: dict, kind: str | None) -> dict:
    m = meta(obj)
    ref = {
        "kind": kind or obj.get("kind", ""),
        "namespace": m.get("namespace", ""),
        "name": m.get("name", ""),
        "uid": m.get("uid", ""),
        "apiVersion": obj.get("apiVersion", ""),
        "resourceVersion": m.get("resourceVersion", ""),
    }
    if not ref["apiVersion"] and ref["kind"]:
        try:
            ref["apiVersion"] = R.by_kind(ref["kind"]).api_version
        except KeyError:
            pass
    return ref


def _blocked_key(obj: dict, kind: str | None):
    """The spam filter's shortcut key for an object: its UID (one object incarnation, whatever its kind), or
    kind, apiVersion, namespace and name for an object without one."""
    m = obj.get("metadata") or {}
    uid = m.get("uid")
    if uid:
        return uid
    return kind or obj.get("kind", ""), obj.get("apiVersion", ""), m.get("namespace", ""), m.get("name", "")


class BroadcastRecorder(EventRecorder):
    """Asynchronous recorder with the client-go correlator, writing Events through `client`."""

    def __init__(self, client: KubeClient, component: str = C.CONTROLLER_AGENT_NAME, *, spam_filter: bool = True,
                 log_events: bool = True, writers: int = 1, coalesce: bool = False, repeat_window: float = 0.0,
                 cache_limit=CACHE_LIMIT):
        self.client = client
        # correlator cache size: client-go's 4096 (an int), or a callable re-read when a cache is trimmed —
        # native mode sizes it to the objects the controller manages, so a repeat stays a count PATCH
        # instead of becoming a new Event once more than 4096 objects emit events
        self.cache_limit = cache_limit
        self.component = component
        self.spam_filter = spam_filter
        self.log_events = log_events
        # client-go writes through one sink goroutine; with `writers` > 1 events are spread over that many
        # writer tasks by involved object, so each object's events (and their dedup PATCHes) stay ordered
        self.writers = max(1, writers)
        self._queues: list[asyncio.Queue] = [asyncio.Queue(maxsize=max(1, BUFFER // self.writers))
                                             for _ in range(self.writers)]
        self._queue = self._queues[0]
        self.coalesce = coalesce
        self._pending: dict[tuple, list] = {}  # coalesce: correlation key -> queued entry [.., n]
        self.repeat_window = repeat_window if coalesce else 0.0
        self._deferred: dict[tuple, list] = {}  # repeat_window: correlation key -> held entry [.., n]
        self._flush_timer = None
        self._buckets: dict[tuple, TokenBucket] = {}
        self._blocked: dict[tuple, float] = {}  # (kind, apiVersion, ns, name, uid) -> when its next token is due
        self._similar: dict[tuple, tuple[set, float]] = {}  # aggregate key -> (messages, first_seen)
        self._seen: dict[tuple, list] = {}  # full key -> [name, count] of the Event last written
        self._tasks: list[asyncio.Task] = []
        self._write_meta = getattr(client, "write_meta", None)  # undecoded writes (REST clients)
        self.stats = {"recorded": 0, "dropped_spam": 0, "dropped_full": 0, "created": 0, "patched": 0, "failed": 0,
                      "merged": 0, "warnings_held": 0}

    def start(self) -> None:
        if not self._tasks:
            self._tasks = [asyncio.ensure_future(self._run(q)) for q in self._queues]

    async def stop(self, drain_timeout: float = 1.0) -> None:
        if self._flush_timer is not None:
            self._flush_timer.cancel()
            self._flush_timer = None
        if self._deferred and self._tasks:
            for entry in self._deferred.values():  # held repeats still go out (up to the buffers' room)
                self._enqueue(entry, held=True)
            self._deferred.clear()
        if not self._tasks:
            return
        try:
            await wait_timeout(asyncio.gather(*(q.join() for q in self._queues)), drain_timeout)
        except asyncio.TimeoutError:
            pass
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):  # noqa: BLE001
                pass
        self._tasks = []

    def event(self, obj, event_type, reason, message, kind=None):
        self.stats["recorded"] += 1
        blocked = self._blocked
        if blocked and not (self.log_events and log.isEnabledFor(logging.INFO)):
            # an object whose spam bucket is empty: dropped before its reference is built (the bucket's
            # refill is linear, so skipping its update until the next token is due changes nothing)
            until = blocked.get(_blocked_key(obj, kind))
            if until is not None and time.monotonic() < until:
                self.stats["dropped_spam"] += 1
                return
        ref = involved_object(obj, kind)
        if self.log_events and log.isEnabledFor(logging.INFO):
            log.info("Event occurred", extra={"object": f"{ref['namespace']}/{ref['name']}", "kind": ref["kind"],
                                              "type": event_type, "reason": reason, "message": message})
        now = time.monotonic()
        if not self._allow(ref, now):
            self.stats["dropped_spam"] += 1
            b = self._buckets.get((self.component, ref["kind"], ref["namespace"], ref["name"], ref["uid"],
                                   ref["apiVersion"]))
            if b is not None and b.qps > 0:
                blocked[_blocked_key(obj, kind)] = now + (1.0 - b._tokens) / b.qps
                _bound(blocked, self.cache_limit)
            return
        message, key = self._aggregate(ref, event_type, reason, message, now)
        if self.coalesce:
            entry = self._pending.get(key) or self._deferred.get(key)
            if entry is not None:
                entry[4] += 1
                entry[0], entry[3] = ref, message  # the latest involvedObject and message go out with the write
                self.stats["merged"] += 1
                return
            if self.repeat_window > 0 and key in self._seen:
                # a repeat of an Event already written: held, and folded with those that follow it
                self._deferred[key] = [ref, event_type, reason, message, 1, key]
                if self._flush_timer is None:
                    self._flush_timer = asyncio.get_running_loop().call_later(self.repeat_window,
                                                                              self._flush_deferred)
                return
        self._enqueue([ref, event_type, reason, message, 1, key])

    def _flush_deferred(self) -> None:
        """Hand the held repeats to the writers — as many as their buffers take now (a held repeat is never
        dropped for a full buffer: the rest waits for the next, short, round)."""
        self._flush_timer = None
        room = sum(q.maxsize - q.qsize() for q in self._queues)
        for key in list(self._deferred)[:max(0, room)]:
            if self._enqueue(self._deferred[key], held=True):
                del self._deferred[key]
        if self._deferred:
            self._flush_timer = asyncio.get_running_loop().call_later(0.01, self._flush_deferred)

    def _enqueue(self, entry: list, held: bool = False) -> bool:
        """Queue for its object's writer; False when that buffer is full (a new event is then dropped, as
        client-go drops on a full broadcaster buffer; a held repeat stays held).  With coalescing (native
        mode) a Warning is not dropped for a full buffer: it waits in the held set and goes out with the
        next flush — a burst of `Synced` Events must not swallow the one that reports a failure."""
        ref, key = entry[0], entry[5]
        q = self._queue if self.writers == 1 else \
            self._queues[hash((ref["namespace"], ref["name"], ref["kind"])) % self.writers]
        if held and q.full():
            return False
        try:
            q.put_nowait(entry)
        except asyncio.QueueFull:
            if self.coalesce and entry[1] == C.EVENT_TYPE_WARNING and len(self._deferred) < WARNING_OVERFLOW:
                self._deferred[key] = entry
                self.stats["warnings_held"] += 1
                if self._flush_timer is None:
                    self._flush_timer = asyncio.get_running_loop().call_later(0.01, self._flush_deferred)
                return False
            self.stats["dropped_full"] += 1
            return False
        if self.coalesce:
            self._pending[key] = entry
        return True

    # ------------------------------------------------------------------ correlator
    def _allow(self, ref: dict, now: float) -> bool:
        if not self.spam_filter:
            return True
        k = (self.component, ref["kind"], ref["namespace"], ref["name"], ref["uid"], ref["apiVersion"])
        b = self._buckets.get(k)
        if b is None:
            b = self._buckets[k] = TokenBucket(SPAM_QPS, SPAM_BURST, now=now)
            _bound(self._buckets, self.cache_limit)
        return b.reserve(now) <= 0.0 or self._refund(b)

    @staticmethod
    def _refund(b: TokenBucket) -> bool:
        b._tokens += 1.0  # a rejected event must not consume future capacity (TokenBucket.TryAccept)
        return False

    def _aggregate(self, ref: dict, event_type: str, reason: str, message: str, now: float) -> tuple[str, tuple]:
        akey = (self.component, ref["kind"], ref["namespace"], ref["name"], ref["uid"], event_type, reason)
        hit = self._similar.get(akey)
        if hit is None or now - hit[1] > AGGREGATE_INTERVAL_S:
            hit = self._similar[akey] = (set(), now)
            _bound(self._similar, self.cache_limit)
        msgs = hit[0]
        msgs.add(message)
        if len(msgs) >= AGGREGATE_MAX_EVENTS:
            return "(combined from similar events): " + message, akey
        return message, akey + (message,)

    async def _write(self, ref, event_type, reason, message, n: int, key: tuple) -> None:
        """One sink write for `n` correlated occurrences of an event (n > 1 only when coalescing)."""
        ts = now_rfc3339()
        prev = self._seen.get(key)
        ns = ref["namespace"] or "default"
        wm = self._write_meta
        if prev is not None:  # [name, count]: only these matter for the count PATCH
            count = prev[1] + n
            patch = {"count": count, "lastTimestamp": ts, "message": message}
            if wm is not None:  # skip decoding the response
                await wm("patch", R.EVENTS, ns, patch, name=prev[0], patch_type=PATCH_STRATEGIC)
            else:
                res = await self.client.patch(R.EVENTS, ns, prev[0], patch, patch_type=PATCH_STRATEGIC)
                if isinstance(res, dict):
                    count = int(res.get("count", count))
            prev[1] = count
            self.stats["patched"] += 1
            return
        ev = {
            "apiVersion": "v1",
            "kind": "Event",
            "metadata": {"name": f"{ref['name']}.{time.time_ns():x}", "namespace": ns},
            "involvedObject": ref,
            "reason": reason,
            "message": message,
            "source": {"component": self.component},
            "firstTimestamp": ts,
            "lastTimestamp": ts,
            "count": n,
            "type": event_type,
            "reportingComponent": self.component,
            "reportingInstance": "",
        }
        if wm is not None:
            await wm("create", R.EVENTS, ns, ev)
            res = None
        else:
            res = await self.client.create(R.EVENTS, ns, ev)
        done = res if isinstance(res, dict) else ev
        self._seen[key] = [(done.get("metadata") or {}).get("name", ev["metadata"]["name"]),
                           int(done.get("count", n))]
        _bound(self._seen, self.cache_limit)
        self.stats["created"] += 1

    async def _run(self, queue: asyncio.Queue) -> None:
        while True:
            entry = await queue.get()
            if self.coalesce and self._pending.get(entry[5]) is entry:
                del self._pending[entry[5]]  # from here on, a repeat queues a write of its own
            ref, event_type, reason, message, n, key = entry
            try:
                for attempt in range(3):
                    try:
                        await self._write(ref, event_type, reason, message, n, key)
                        break
                    except asyncio.CancelledError:
                        raise
                    except Exception as e:  # noqa: BLE001
                        if attempt == 2:
                            self.stats["failed"] += 1
                            log.warning("unable to write event: %r", e)
                        else:
                            await asyncio.sleep(0.1 * (attempt + 1))
            finally:
                queue.task_done()
