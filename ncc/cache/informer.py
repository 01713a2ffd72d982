"""SharedInformer: list → watch → resync, feeding a `Store` and fanning out to handlers.

Re-creates the client-go machinery the reference gets from
`SharedInformerFactory(..., 30s, WithNamespace(ns))` (main.go:70-71):

* initial (paginated) LIST → `Store.replace` → `has_synced()` becomes true;
* WATCH from the list resourceVersion with bookmarks; a clean stream end re-watches from the
  last seen RV; `410 Gone` (HTTP or in-stream ERROR) triggers a relist;
* transport errors back off exponentially (client-go's 800ms→30s reflector backoff);
* a relist delivers Add for new keys, Update for kept keys, and Delete with a
  `DeletedFinalStateUnknown` tombstone for keys that vanished while we were not watching;
* every `resync_period` seconds each cached object is re-delivered as Update(obj, obj),
  which is what makes the reference re-reconcile every template every 30 s
  (controller.go:288-290).

Handlers run inline on the event loop; a handler may be a coroutine function, in which case
the informer awaits it before processing the next event (the reference's template-delete
handler blocks its informer the same way, controller.go:195-205).
"""
from __future__ import annotations

import asyncio
import inspect
import logging
import random
from dataclasses import dataclass
from typing import Callable

from .. import native as _native
from ..aio import wait_timeout
from ..api.jsonenc import dumps_bytes, loads_fast
from ..api.objects import ObjectKey, key_of, rv_int
from ..api.resources import ResourceType
from ..kube import errors as E
from ..kube.client import KubeClient
from .store import Store

log = logging.getLogger("ncc.informer")
_UNREADABLE = (ValueError, AttributeError, TypeError)  # a relayed line that is not a JSON watch event


@dataclass(frozen=True)
class DeletedFinalStateUnknown:
    """Tombstone for an object whose delete event was missed (client-go cache.DeletedFinalStateUnknown)."""
    key: ObjectKey
    obj: dict


class Lister:
    """Namespace-aware read view over a store; `get` raises `NotFound` like a client-go lister."""

    def __init__(self, store: Store, rt: ResourceType):
        self.store = store
        self.rt = rt

    def get(self, namespace: str, name: str) -> dict:
        o = self.store.get(namespace, name)
        if o is None:
            gr = f"{self.rt.plural}.{self.rt.group}" if self.rt.group else self.rt.plural
            raise E.NotFound(f'{gr} "{name}" not found', details={"name": name, "kind": self.rt.plural})
        return o

    def try_get(self, namespace: str, name: str) -> dict | None:
        return self.store.get(namespace, name)

    def list(self, namespace: str | None = None) -> list[dict]:
        return self.store.list(namespace)


_OBJECT_EVENTS = frozenset(("ADDED", "MODIFIED", "DELETED"))


@dataclass
class _Handler:
    on_add: Callable | None
    on_update: Callable | None
    on_delete: Callable | None


async def _single_lines(lines):
    """Adapt a line-at-a-time raw watch to the batched loop."""
    async for line in lines:
        yield (line,)


class Informer:
    def __init__(self, client: KubeClient, rt: ResourceType, namespace: str | None, *,
                 resync_period: float = 0.0, transform: Callable[[dict], dict] | None = None,
                 label_selector: str | None = None, page_size: int = 500, watch_timeout: tuple = (300, 600),
                 name: str = "", key_filter: Callable[[str, str], bool] | None = None,
                 owner_filter: Callable[[str, str, tuple], bool] | None = None):
        self.client = client
        # key_filter(ns, name) / owner_filter(ns, name, owner_names) → False drops the object before it is
        # decoded/stored (a partitioned executor skips the other partitions' templates, and dependents
        # owned only by them, straight off the wire via the native scanner).  An object that leaves the
        # filter (e.g. our ownerRef removed) is dropped from the store.
        self.key_filter = key_filter
        self.owner_filter = owner_filter
        self.filtered = 0
        # Writes in flight (`begin_write`/`end_write`): a watch event for such a key may overtake the
        # write's HTTP response.  It is parked undecoded and, once the response is in, dropped if it is
        # the write's own echo — the common case — or applied if it is someone else's newer version.
        self._inflight: dict = {}
        self._stash: dict = {}
        self._owner_sigs: dict = {}  # key -> (cached object, owner names, owner uids): the metadata-only filter
        self._owner_memo = None  # the native metadata-only filter with its memo (native/ext/scan.hpp OwnerFilter)
        # set by the owner when the apiserver answers its other requests again (ncc/shards/shard.py): a
        # list/watch waiting out an outage backoff retries at once, once per outage
        self.answering: asyncio.Event | None = None
        self.watching = False  # a watch request is open (executor status)
        # metadata_only: the consumer needs names/ownerReferences, never payloads (the coordinator's view
        # of Secrets/ConfigMaps).  MODIFIED events that leave the owner list unchanged are skipped without
        # decoding; stored objects keep metadata only.
        self.metadata_only = False
        self.rt = rt
        self.namespace = namespace
        self.resync_period = resync_period
        self.label_selector = label_selector
        self.page_size = page_size
        self.watch_timeout = watch_timeout
        self.name = name or f"{client.cluster_name}/{rt.plural}"
        self.store = Store(transform=transform)
        self.lister = Lister(self.store, rt)
        self._handlers: list[_Handler] = []
        self._synced = asyncio.Event()
        self._task: asyncio.Task | None = None
        self._resync_task: asyncio.Task | None = None
        self.last_rv: str = ""
        self.relists = 0
        self.events = 0
        self.last_error: BaseException | None = None
        self._stopping = False
        # Echo fast path: when this informer's store receives assumed write results (mutation overlay),
        # watch events for exactly those versions are recognised by the native scanner from the raw line
        # and promoted without json decoding or handler dispatch (the writer already acted on them).
        self.echo_fastpath = False
        self.echoes = 0
        # Watch relay (ncc/controller/relay.py): `tap` sees every raw line and listing this informer takes in
        # (the coordinator forwarding them); `feed` replaces LIST/WATCH by what a coordinator forwards.
        self.tap = None
        self.feed = None
        # Optional native decoder for watch lines returning (type, object) or None (then the full decode):
        # the coordinator's template informer keeps slim templates (`_native.template_event_slim`; called as
        # slim_decode(line, store items, default namespace) so unchanged parts come from the cached version).
        self.slim_decode = None

    # ------------------------------------------------------------- public API
    def add_event_handler(self, on_add=None, on_update=None, on_delete=None) -> None:
        self._handlers.append(_Handler(on_add, on_update, on_delete))

    def has_synced(self) -> bool:
        return self._synced.is_set()

    async def wait_for_sync(self, timeout: float | None = None) -> bool:
        try:
            await wait_timeout(self._synced.wait(), timeout)
            return True
        except asyncio.TimeoutError:
            return False

    def start(self) -> asyncio.Task:
        if self._task is None:
            self._task = asyncio.ensure_future(self._run())
            if self.resync_period > 0:
                self._resync_task = asyncio.ensure_future(self._resync_loop())
        return self._task

    async def stop(self) -> None:
        self._stopping = True
        for t in (self._task, self._resync_task):
            if t is not None:
                t.cancel()
        pending = [t for t in (self._task, self._resync_task) if t is not None]
        if pending:
            await asyncio.wait(pending, timeout=5.0)
        self._task = self._resync_task = None

    # ------------------------------------------------------------- dispatch
    # handlers are plain callables; one that returns an awaitable (e.g. the reference-compat inline delete)
    # is awaited before the next event, like client-go's serial handler delivery
    async def _dispatch_add(self, obj):
        for h in self._handlers:
            fn = h.on_add
            if fn is not None:
                r = fn(obj)
                if r is not None and inspect.isawaitable(r):
                    await r

    async def _dispatch_update(self, old, new):
        for h in self._handlers:
            fn = h.on_update
            if fn is not None:
                r = fn(old, new)
                if r is not None and inspect.isawaitable(r):
                    await r

    async def _dispatch_delete(self, obj):
        for h in self._handlers:
            fn = h.on_delete
            if fn is not None:
                r = fn(obj)
                if r is not None and inspect.isawaitable(r):
                    await r

    # ------------------------------------------------------------- reflector
    async def _list(self, resource_version: str | None = None) -> str:
        """LIST (paginated).  Like client-go's reflector, the first page asks for `resourceVersion` — "0" on
        a cold start, i.e. anything the apiserver's watch cache holds, instead of a quorum read of every page
        from etcd; "" (consistent) after the watch expired (410 Gone)."""
        items: list[dict] = []
        token = None
        rv = ""
        tap = self.tap
        paged_tap = getattr(tap, "on_list_page", None)
        transform = self.store.transform
        while True:
            resp = await self.client.list(self.rt, self.namespace, label_selector=self.label_selector,
                                          limit=self.page_size, continue_token=token,
                                          resource_version=resource_version if token is None else None)
            page = resp.get("items") or []
            # Each page goes to the relay (full objects: executors need the specs) and into its stored form at
            # once, so a listing holds one page of full objects at a time, not all of them: at 10 000 templates
            # with their Secrets and ConfigMaps that is the coordinator's start-up and relist peak
            # (bench/suite.py config 4).
            if paged_tap is not None:
                paged_tap(page)
            elif tap is not None:
                items.extend(page)
                page = None
            if page is not None:
                if self.slim_decode is not None:
                    page = self._slim_listing(page)
                elif transform is not None:
                    page = [transform(o) for o in page]
                items.extend(page)
            lm = resp.get("metadata") or {}
            rv = lm.get("resourceVersion", rv)
            token = lm.get("continue")
            if not token:
                break
        if paged_tap is not None:
            tap.on_list(None)  # the listing is complete: the relay swaps it in and sends the snapshots
        elif tap is not None:
            tap.on_list(items)
            if self.slim_decode is not None:
                items = self._slim_listing(items)
            elif transform is not None:
                items = [transform(o) for o in items]
        await self._replace_items(items, transformed=True)
        return rv

    def _slim_listing(self, items: list) -> list:
        """A listing in the form the watch path stores (`slim_decode`): without this the coordinator keeps every
        template's full spec after a LIST — its cold start, and again after each relist — until that template's
        next watch event (the 10 000-template relist storm of bench/suite.py config 4 took its resident set
        from 341 to 563 MiB).  Each item goes through the same native slimming as a watch line."""
        slim, cur, ns = self.slim_decode, self.store._items, self.namespace or ""
        out = []
        for o in items:
            try:
                sl = slim(b'{"type":"ADDED","object":' + dumps_bytes(o) + b"}", cur, ns)
            except (TypeError, ValueError):
                sl = None
            out.append(sl[1] if sl is not None else o)
        return out

    async def _replace_items(self, items: list, transformed: bool = False) -> None:
        """Swap in a complete listing (LIST, or a relayed snapshot) and deliver the differences.  `transformed`:
        the items are already in stored form (`Store.transform` applied)."""
        if self.key_filter is not None or self.owner_filter is not None:
            items = [o for o in items if self._wanted(o.get("metadata") or {})]
        self._stash.clear()  # the relist is newer than anything parked
        if self._owner_memo is not None:
            self._owner_memo.clear()  # it holds the versions it compared against: not past a relist
        added, updated, deleted = self.store.replace(items, transformed=transformed)
        self.relists += 1
        synced_before = self.has_synced()
        self._synced.set()
        for o in added:
            await self._dispatch_add(o)
        for old, new in updated:
            await self._dispatch_update(old, new)
        if synced_before:
            for o in deleted:
                await self._dispatch_delete(DeletedFinalStateUnknown(key_of(o), o))

    def _line_ctx(self, force: bool = False):
        """Scanner state for the raw-line path, or None when lines must be decoded one by one (no native
        module, or nothing to gain: no filters, no echo promotion, no metadata-only skipping).  `force`
        asks for the raw path whenever the native module is there (a relayed feed is raw lines anyway)."""
        kf, of = self.key_filter, self.owner_filter
        mo = self.metadata_only
        if not (force or self.echo_fastpath or kf is not None or of is not None or mo or self.slim_decode):
            return None
        mod = _native.load()
        if mod is None:
            return None
        scan = mod.scan_event_owners if (of is not None or mo) else mod.scan_event
        nparts = 0
        kpart = opart = oref = None
        # partition filters (executor key partitions) are evaluated natively: crc32 % parts of the key and
        # of every owner, so a foreign line costs one scan and two integer tests
        parts = {getattr(f, "parts", None) for f in (kf, of) if f is not None}
        if len(parts) == 1 and None not in parts:
            nparts = parts.pop()
            default_ns_ = self.namespace or ""

            def scan(line, _s=mod.scan_event_part, _p=nparts, _d=default_ns_):
                return _s(line, _p, _d)
            kpart = kf.part if kf is not None else None
            opart = of.part if of is not None else None
            oref = getattr(of, "referenced", None) if of is not None else None
            kf = of = None
        batch_filter = None
        if mo:
            if self._owner_memo is None and hasattr(mod, "OwnerFilter"):
                self._owner_memo = mod.OwnerFilter()
            batch_filter = self._owner_memo if self._owner_memo is not None else getattr(mod, "owner_filter", None)
        return (scan, nparts, kpart, opart, oref, kf, of, mo, batch_filter)

    async def _watch(self, rv: str) -> str:
        """Consume one watch stream; returns the last RV seen.  Raises Gone to force a relist."""
        lo, hi = self.watch_timeout
        kw = dict(resource_version=rv, timeout_seconds=random.randint(lo, hi), allow_bookmarks=True,
                  label_selector=self.label_selector)
        ctx = self._line_ctx(force=self.tap is not None) if hasattr(self.client, "watch_raw") else None
        if ctx is not None:
            batches = getattr(self.client, "watch_raw_batches", None)
            tap = self.tap
            if batches is not None and tap is not None and getattr(self.client, "supports_line_tap", False):
                # the relay gets every line straight off the socket: an executor is not kept waiting while
                # this coordinator works through the batches before it (docs/BENCHMARKS_ARCHIVE.md, latency stages)
                source = batches(self.rt, self.namespace, on_lines=tap.on_lines, **kw)
                tap = None
            elif batches is not None:
                source = batches(self.rt, self.namespace, **kw)
            else:
                source = _single_lines(self.client.watch_raw(self.rt, self.namespace, **kw))
            async for lines in source:
                if tap is not None:
                    tap.on_lines(lines)
                rv = await self._consume(lines, ctx, rv)
            return rv
        async for ev in self.client.watch(self.rt, self.namespace, **kw):
            rv = await self._handle(ev.type, ev.object, rv)
        return rv

    async def _consume(self, lines, ctx, rv: str) -> str:
        """Apply one batch of raw watch lines (see `_line_ctx`); returns the last RV seen."""
        scan, nparts, kpart, opart, oref, kf, of, mo, _owner_filter = ctx
        loads = loads_fast
        slim = self.slim_decode
        store = self.store
        default_ns = self.namespace or ""
        inflight, stash = self._inflight, self._stash
        sigs = self._owner_sigs
        unfiltered = self.key_filter is None and self.owner_filter is None
        last = None
        if mo and not nparts and kf is None and of is None and _owner_filter is not None:
            # the whole batch through the native owner filter; what it keeps takes the path below
            lines, dropped, last = _owner_filter(lines if type(lines) is list else list(lines), store._items,
                                                 store._assumed, default_ns)
            self.filtered += dropped
        for line in lines:
            sc = None
            if nparts:
                sc = scan(line)
                if sc is not None and sc[0] in _OBJECT_EVENTS and (
                        (kpart is not None and sc[6] != kpart) or
                        (opart is not None and sc[4] and not (sc[7] >> opart) & 1 and
                         (oref is None or not oref(sc[1] or default_ns, sc[2])))):
                    rv = self.last_rv = sc[3]
                    self._filtered_out(sc[1] or default_ns, sc[2])
                    continue
            elif kf is not None or of is not None:
                sc = scan(line)
                if sc is not None and sc[0] in _OBJECT_EVENTS:
                    ns_ = sc[1] or default_ns
                    if (kf is not None and not kf(ns_, sc[2])) or \
                            (of is not None and not of(ns_, sc[2], sc[4])):
                        rv = self.last_rv = sc[3]
                        self._filtered_out(ns_, sc[2])
                        continue
            if mo:
                if sc is None:
                    sc = scan(line)
                if sc is not None and sc[0] == "MODIFIED":
                    k2 = (sc[1] or default_ns, sc[2])
                    cur = store.get(*k2)
                    if cur is not None:
                        # the owners of the cached version, as the scan reports them, kept per key while that
                        # version stays cached (a metadata-only store changes only on an owner change)
                        sig = sigs.get(k2)
                        if sig is None or sig[0] is not cur:
                            if len(sigs) > len(store._items) + 4096:
                                sigs.clear()
                            refs = (cur.get("metadata") or {}).get("ownerReferences") or ()
                            sig = sigs[k2] = (cur, tuple(r.get("name", "") for r in refs),
                                              tuple(r.get("uid", "") for r in refs))
                        if sig[1] == sc[4] and sig[2] == sc[5]:
                            if store._assumed:  # (typically our adoption's echo) the overlay becomes the stored version
                                store.promote(k2, sc[3])
                            rv = self.last_rv = sc[3]
                            self.filtered += 1
                            continue
            if store._assumed or inflight:
                if sc is None:
                    sc = scan(line)
                if sc is not None and sc[0] in ("ADDED", "MODIFIED"):
                    key = ObjectKey(sc[1] or default_ns, sc[2])
                    if store.confirm(key, sc[3]) is not None:
                        rv = self.last_rv = sc[3]
                        self.events += 1
                        self.echoes += 1
                        continue
                    if key in inflight:  # overtook the response of our write: park it
                        prev = stash.get(key)
                        if prev is not None:
                            await self._apply_line(prev[1])
                        stash[key] = (sc[3], line)
                        rv = self.last_rv = sc[3]
                        continue
            if stash and sc is not None:
                prev = stash.pop(ObjectKey(sc[1] or default_ns, sc[2]), None)
                if prev is not None:  # keep per-key order
                    await self._apply_line(prev[1])
            sl = slim(line, store._items, default_ns) if slim is not None else None
            if sl is not None:
                if sl[0] == "MODIFIED" and not unfiltered:
                    rv = await self._handle(sl[0], sl[1], rv)
                    continue
                if sl[0] == "MODIFIED":
                    # _handle → _apply → _dispatch_update inlined for the common case (no coroutine per layer)
                    obj = sl[1]
                    self.events += 1
                    stored, old = store.upsert(obj)
                    if old is None:
                        await self._dispatch_add(stored)
                    else:
                        for h in self._handlers:
                            fn = h.on_update
                            if fn is not None:
                                r = fn(old, stored)
                                if r is not None and inspect.isawaitable(r):
                                    await r
                    rv = self.last_rv = (obj.get("metadata") or {}).get("resourceVersion") or rv
                    continue
                rv = await self._handle(sl[0], sl[1], rv)
                continue
            ev = loads(line)
            rv = await self._handle(ev.get("type", ""), ev.get("object") or {}, rv)
        if last is not None:  # the batch ended with a dropped line
            rv = self.last_rv = last
        return rv

    async def _handle(self, t: str, obj: dict, rv: str) -> str:
        if t == "ERROR":
            code = int(obj.get("code") or 0)
            if code == 410:
                raise E.Gone(obj.get("message", "watch expired"))
            raise E.from_status(code, obj)
        new_rv = (obj.get("metadata") or {}).get("resourceVersion") or rv
        if t == "BOOKMARK":
            return new_rv
        if (self.key_filter is not None or self.owner_filter is not None) and t in _OBJECT_EVENTS:
            m = obj.get("metadata") or {}
            if not self._wanted(m):
                self._filtered_out(m.get("namespace") or self.namespace or "", m.get("name", ""))
                self.last_rv = new_rv
                return new_rv
        await self._apply(t, obj)
        self.last_rv = new_rv
        return new_rv

    def _wanted(self, m: dict) -> bool:
        ns = m.get("namespace") or self.namespace or ""
        if self.key_filter is not None and not self.key_filter(ns, m.get("name", "")):
            return False
        if self.owner_filter is not None:
            owners = tuple(r.get("name", "") for r in (m.get("ownerReferences") or ()))
            if not self.owner_filter(ns, m.get("name", ""), owners):
                return False
        return True

    def _filtered_out(self, ns: str, name: str) -> None:
        self.filtered += 1
        if self.store.get(ns, name) is not None:
            self.store.delete(ObjectKey(ns, name))  # left our partition: forget it (no handler dispatch)

    async def _apply_line(self, line: bytes) -> None:
        sl = self.slim_decode(line, self.store._items, self.namespace or "") if self.slim_decode is not None else None
        if sl is not None:
            await self._apply(sl[0], sl[1])
            return
        ev = loads_fast(line)
        await self._apply(ev.get("type", ""), ev.get("object") or {})

    # ------------------------------------------------------------- write tracking
    def begin_write(self, key: ObjectKey) -> None:
        self._inflight[key] = self._inflight.get(key, 0) + 1

    async def end_write(self, key: ObjectKey, obj: dict | None, transformed: bool = False) -> None:
        """Publish a write result (mutation overlay) and settle a parked watch event for the key."""
        n = self._inflight.get(key, 0) - 1
        if n > 0:
            self._inflight[key] = n
        else:
            self._inflight.pop(key, None)
        if obj is not None:
            self.store.assume(obj, transformed)
        if n > 0:
            return
        parked = self._stash.pop(key, None)
        if parked is None:
            return
        if obj is not None:
            prv, orv = rv_int(parked[0]), rv_int((obj.get("metadata") or {}).get("resourceVersion"))
            if prv <= orv:  # our own echo (==) or an older version our write superseded (<)
                if prv == orv and self.store.confirm(key, parked[0]) is not None:
                    self.events += 1
                    self.echoes += 1
                return
        await self._apply_line(parked[1])

    async def _apply(self, t: str, obj: dict) -> None:
        self.events += 1
        if t in ("ADDED", "MODIFIED"):
            stored, old = self.store.upsert(obj)
            if old is None:
                await self._dispatch_add(stored)
            else:
                await self._dispatch_update(old, stored)
        elif t == "DELETED":
            old = self.store.delete(obj)
            await self._dispatch_delete(old if old is not None else obj)

    async def _run_feed(self) -> None:
        """Relay mode (an executor under a coordinator's watch relay, ncc/controller/relay.py): the
        coordinator is the only process listing and watching the controller cluster; it forwards a snapshot
        of every kind once (and again after each of its relists) and then the raw watch lines this
        executor's key partition needs."""
        ctx = self._line_ctx(force=True)
        feed = self.feed
        while not self._stopping:
            what, lines = await feed.get()
            if what == "s":
                loads = loads_fast
                items = []
                for line in lines:
                    try:
                        ev = loads(line)
                        ev.get("type")
                    except (ValueError, AttributeError) as e:
                        log.error("%s: unreadable relayed line skipped: %s", self.name, e)
                        continue
                    if ev.get("type") in ("ADDED", "MODIFIED"):
                        items.append(ev.get("object") or {})
                await self._replace_items(items)
                continue
            try:
                await self._feed_lines(lines, ctx)
            except _UNREADABLE:
                # an unreadable line costs that object, not the rest of its batch: again line by line
                for line in lines:
                    try:
                        await self._feed_lines([line], ctx)
                    except _UNREADABLE as e:
                        log.error("%s: unreadable relayed line skipped: %s", self.name, e)

    async def _feed_lines(self, lines: list, ctx) -> None:
        if ctx is not None:
            self.last_rv = await self._consume(lines, ctx, self.last_rv)
            return
        for line in lines:
            ev = loads_fast(line)
            self.last_rv = await self._handle(ev.get("type", ""), ev.get("object") or {}, self.last_rv)

    async def _run(self) -> None:
        if self.feed is not None:
            await self._run_feed()
            return
        backoff = 0.8
        rv = ""
        need_list = True
        woken = False
        list_rv = "0"  # cold start: served from the apiserver's watch cache
        while not self._stopping:
            try:
                if need_list:
                    rv = await self._list(list_rv)
                    self.last_rv = rv
                    need_list = False
                self.watching = True
                self.last_error = None
                try:
                    rv = await self._watch(self.last_rv or rv)  # resume after the last event we processed
                finally:
                    self.watching = False
                backoff = 0.8
                woken = False
            except asyncio.CancelledError:
                raise
            except E.Gone:
                need_list = True
                list_rv = ""  # our resourceVersion is too old for the cache: consistent read
                log.debug("%s: watch expired, relisting", self.name)
            except Exception as e:  # noqa: BLE001 — transport errors, 5xx, etc.
                self.last_error = e
                log.debug("%s: list/watch failed: %r; retry in %.2fs", self.name, e, backoff)
                wait = backoff * (1 + random.random() * 0.2)
                outage = isinstance(e, E.TransportError) or (isinstance(e, E.ApiError) and (e.code or 0) >= 500)
                ans = self.answering
                if outage and ans is not None and not woken:
                    ans.clear()  # the owner's next answered request ends the wait (once per outage)
                    try:
                        await asyncio.wait_for(ans.wait(), wait)
                        woken = True
                    except asyncio.TimeoutError:
                        pass
                else:
                    await asyncio.sleep(wait)
                backoff = min(backoff * 2, 30.0)
                if not isinstance(e, E.TransportError):
                    need_list = True
                    list_rv = self.last_rv or "0"  # not older than what we have seen

    async def _resync_loop(self) -> None:
        while True:
            await asyncio.sleep(self.resync_period)
            if not self.has_synced():
                continue
            for o in self.store.list():
                await self._dispatch_update(o, o)


class InformerFactory:
    """One informer per resource type for one (client, namespace) — SharedInformerFactory analogue."""

    def __init__(self, client: KubeClient, namespace: str | None, resync_period: float = 0.0, **informer_kw):
        self.client = client
        self.namespace = namespace
        self.resync_period = resync_period
        self.informer_kw = informer_kw
        self._informers: dict[ResourceType, Informer] = {}

    def informer(self, rt: ResourceType, **kw) -> Informer:
        inf = self._informers.get(rt)
        if inf is None:
            opts = dict(self.informer_kw)
            opts.update(kw)
            inf = self._informers[rt] = Informer(self.client, rt, self.namespace,
                                                 resync_period=self.resync_period, **opts)
        return inf

    def start(self) -> None:
        for inf in self._informers.values():
            inf.start()

    async def stop(self) -> None:
        for inf in self._informers.values():
            await inf.stop()

    def has_synced(self) -> bool:
        return all(i.has_synced() for i in self._informers.values())

    async def wait_for_sync(self, timeout: float | None = None) -> bool:
        res = await asyncio.gather(*(i.wait_for_sync(timeout) for i in self._informers.values()))
        return all(res)

    def informers(self) -> list[Informer]:
        return list(self._informers.values())
