"""Watch relay: the coordinator is the only process that lists and watches the controller cluster.

The reference runs one namespace-scoped informer factory per cluster (main.go:70-71): every kind is
listed once and watched over one stream.  Native mode runs k executors per shard group × N groups;
if each of them listed and watched the controller cluster itself, that cluster would serve
1 + N·k LIST+WATCH streams per kind, and a 410 relist would cost N·k full LISTs.

Instead the coordinator's four controller informers get a *tap* (`Informer.tap`): every raw watch
line and every listing they take in is forwarded, undecoded, over the executors' existing
socketpairs (`ncc.controller.ipc`):

* `{"t": "s", "k": kind, "l": [line, ...]}` — snapshot of one kind (after the coordinator's LIST
  and after each relist; and to every executor when it (re)starts), as `ADDED` watch lines;
* `{"t": "w", "k": kind, "l": [line, ...]}` — raw watch lines as they arrive.

Lines are routed by key partition, computed natively (`_native.relay_scan`): a template or
workgroup goes to the executors of its key partition (one per shard group); a Secret/ConfigMap to
the partitions of its owner templates and of the templates referencing it (the coordinator's
reverse index), and to every executor while it has no owner.  With one executor per shard group no
routing is needed.  The executor side (`Informer.feed`) applies snapshots and lines exactly like a
LIST and a watch stream — the Python executor through the same informer code, the C++ executor
(`native/executor/`) through its own cache.

Result: the controller apiserver serves one LIST + one WATCH per kind per coordinator, whatever the
number of shards and executors.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time
from collections import deque

import msgpack

from .. import native as _native
from ..api import resources as R
from ..api.jsonenc import dumps_bytes
from ..api.objects import meta

log = logging.getLogger("ncc.relay")

KINDS = (R.TEMPLATES, R.WORKGROUPS, R.SECRETS, R.CONFIGMAPS)
_DEP_INDEX = {2: "secret", 3: "configmap"}


class RelayFeed:
    """Executor side: the queue an informer in relay mode consumes (`Informer.feed`)."""
    __slots__ = ("_items", "_waiter", "partial")

    def __init__(self):
        self._items: deque = deque()
        self._waiter: asyncio.Future | None = None
        self.partial: list = []  # lines of a chunked snapshot still arriving

    def put(self, what: str, lines: list) -> None:
        self._items.append((what, lines))
        w = self._waiter
        if w is not None:
            self._waiter = None
            if not w.done():
                w.set_result(None)

    async def get(self) -> tuple:
        while not self._items:
            fut = self._waiter = asyncio.get_running_loop().create_future()
            try:
                await fut
            finally:
                if self._waiter is fut:
                    self._waiter = None
        return self._items.popleft()


def deliver(feeds: list, msg: dict) -> bool:
    """Executor side: hand a relay message to the feed of its kind; False if `msg` is no relay message.  A
    listing that came in chunks (all but the last with "more") is handed over whole, as one snapshot."""
    t = msg.get("t")
    if t not in ("s", "w"):
        return False
    feed = feeds[msg["k"]]
    if t == "s":
        if msg.get("more"):
            feed.partial.extend(msg["l"])
            return True
        if feed.partial:
            lines, feed.partial = feed.partial + list(msg["l"]), []
            feed.put("s", lines)
            return True
    feed.put(t, msg["l"])
    return True


SNAPSHOT_CHUNK = 4 << 20  # bytes of watch lines per snapshot message (frames stay far below ipc.MAX_FRAME)


def snapshot_messages(kind: int, lines: list, chunk: int | None = None) -> list:
    """A listing as relay messages of at most ~`chunk` bytes each ("more" on all but the last)."""
    chunk = SNAPSHOT_CHUNK if chunk is None else chunk
    out, cur, size = [], [], 0
    for line in lines:
        if cur and size + len(line) > chunk:
            out.append({"t": "s", "k": kind, "l": cur, "more": True})
            cur, size = [], 0
        cur.append(line)
        size += len(line)
    out.append({"t": "s", "k": kind, "l": cur})
    return out


class _Tap:
    __slots__ = ("relay", "kind")

    def __init__(self, relay: "WatchRelay", kind: int):
        self.relay, self.kind = relay, kind

    def on_list(self, items: list | None) -> None:
        self.relay.on_list(self.kind, items)

    def on_list_page(self, items: list) -> None:
        self.relay.on_list_page(self.kind, items)

    def on_lines(self, lines: list) -> None:
        self.relay.on_lines(self.kind, lines)


def _line_of(obj: dict) -> bytes:
    return b'{"type":"ADDED","object":' + dumps_bytes(obj) + b"}"


class WatchRelay:
    """Coordinator side.  `informers` are the coordinator's controller informers in `KINDS` order;
    `template_store` carries the "secret"/"configmap" reverse indices (native mode)."""

    def __init__(self, informers: list, template_store, namespace: str):
        self.namespace = namespace or ""
        self.template_store = template_store
        self.raw: list[dict] = [{} for _ in KINDS]  # (ns, name) -> latest line of the object
        self._listing: dict[int, dict] = {}  # kind -> lines of a listing still arriving page by page
        self._index: list = [None] * len(KINDS)  # per kind, the native one-partition index loop (RelayIndex)
        self.synced = [False] * len(KINDS)
        self.handles: list = []
        self.parts = 1
        self._by_part: dict[int, list] = {}
        self._mod = _native.load()
        self.stats = {"lines_in": 0, "lines_out": 0, "snapshots": 0, "frames": 0}
        # NCC_TRACE_STAGES=<dir>: record when each watch line was relayed (bench.py --stages joins it with the
        # apiservers' commit times and the executors' receive/dequeue times: where does an object's latency go?)
        self.trace: list | None = [] if os.environ.get("NCC_TRACE_STAGES") else None
        for k, inf in enumerate(informers):
            inf.tap = _Tap(self, k)

    # ------------------------------------------------------------------ executors
    def attach(self, handle) -> None:
        """An executor (re)started: its channel gets a snapshot of every kind synced so far, then live lines."""
        if handle not in self.handles:
            self.handles.append(handle)
        self._reindex()
        for k, ok in enumerate(self.synced):
            if ok:
                self._send_snapshot(k, [handle])

    def on_need(self, handle, msg: dict) -> None:
        """An executor misses a controller object it needs (e.g. a dependent routed elsewhere while another
        partition's template owned it, before one of this partition's templates referenced it): send the
        latest line of it, if the object exists."""
        kind = msg.get("k")
        ns, _, name = str(msg.get("n", "")).partition("/")
        if not isinstance(kind, int) or not 0 <= kind < len(KINDS):
            return
        line = self.raw[kind].get((ns, name))
        if line is not None:
            self._send(handle, {"t": "w", "k": kind, "l": [line]})
            self.stats["needs_served"] = self.stats.get("needs_served", 0) + 1

    def detach(self, handle) -> None:
        if handle in self.handles:
            self.handles.remove(handle)
            self._reindex()

    def _reindex(self) -> None:
        self.parts = max((h.parts for h in self.handles), default=1)
        by: dict[int, list] = {}
        for h in self.handles:
            by.setdefault(h.part, []).append(h)
        self._by_part = by

    # ------------------------------------------------------------------ routing
    def _route(self, kind: int, ns: str, name: str, kp: int, mask: int, n_owners: int) -> int:
        """Bitmask of the key partitions that need this object; -1 = every executor."""
        if kind < 2:
            return 1 << kp
        if not n_owners:
            return -1  # unowned: rogue detection / not yet adopted references need it everywhere
        parts = self.parts
        refs = self.template_store.by_index(_DEP_INDEX[kind], f"{ns}/{name}") if self.template_store else ()
        if refs:
            kpart = self._mod.key_partition
            for t in refs:
                mask |= 1 << kpart(ns, meta(t).get("name", ""), parts)
        return mask

    def _scan(self, line: bytes):
        return self._mod.relay_scan(line, self.parts, self.namespace)

    # ------------------------------------------------------------------ informer side
    def on_list_page(self, kind: int, items: list) -> None:
        """One page of a listing in progress: kept as lines (the objects themselves are not held on to)."""
        ns = self.namespace
        page = self._listing.setdefault(kind, {})
        for o in items:
            page[((meta(o).get("namespace") or ns), meta(o).get("name", ""))] = _line_of(o)

    def on_list(self, kind: int, items: list | None) -> None:
        """A complete listing — `items`, or the pages `on_list_page` collected (None) — replaces the kind's lines
        and goes to every executor as a snapshot."""
        ns = self.namespace
        if items is None:
            self.raw[kind] = self._listing.pop(kind, {})
        else:
            self.raw[kind] = {((meta(o).get("namespace") or ns), meta(o).get("name", "")): _line_of(o) for o in items}
        index = self._index[kind]
        if index is not None and hasattr(index, "clear"):
            index.clear()  # its key tuples are the old dict's: let them go with it (relist-storm peak)
        self.synced[kind] = True
        self._send_snapshot(kind, self.handles)

    def _send_snapshot(self, kind: int, handles: list) -> None:
        if not handles:
            return
        self.stats["snapshots"] += len(handles)
        lines = list(self.raw[kind].values())
        if self.parts <= 1 or self._mod is None:
            for msg in snapshot_messages(kind, lines):
                self._send_all(handles, msg)
            return
        per: dict = {id(h): [] for h in handles}
        for line in lines:
            sc = self._scan(line)
            if sc is None:
                continue
            mask = self._route(kind, sc[1], sc[2], sc[3], sc[4], sc[5])
            for h in handles:
                if mask == -1 or (mask >> h.part) & 1:
                    per[id(h)].append(line)
        for h in handles:
            for msg in snapshot_messages(kind, per[id(h)]):
                self._send(h, msg)

    def on_lines(self, kind: int, lines: list) -> None:
        handles = self.handles
        raw = self.raw[kind]
        mod = self._mod
        if mod is None:
            return
        scan = mod.relay_scan
        parts, ns = self.parts, self.namespace
        self.stats["lines_in"] += len(lines)
        if self.trace is not None:
            now = time.time_ns()
            for line in lines:
                sc = scan(line, 1, ns)
                if sc is not None and sc[0] < 2:
                    self.trace.append((kind, sc[1], sc[2], now))
        if parts <= 1:
            # index + forward in one native call; BOOKMARK / ERROR: the coordinator's informer handles those
            index = self._index[kind]
            if index is None:
                index = self._index[kind] = mod.RelayIndex() if hasattr(mod, "RelayIndex") else mod.relay_index
            keep = index(lines if type(lines) is list else list(lines), raw, ns)
            if keep:
                self._send_all(handles, {"t": "w", "k": kind, "l": keep})
                self.stats["lines_out"] += len(keep) * len(handles)
            return
        per: dict = {}
        by_part = self._by_part
        for line in lines:
            sc = scan(line, parts, ns)
            if sc is None or sc[0] == 3:
                continue
            key = (sc[1], sc[2])
            if sc[0] == 2:
                raw.pop(key, None)
            else:
                raw[key] = line
            mask = self._route(kind, sc[1], sc[2], sc[3], sc[4], sc[5])
            if mask == -1:
                targets = handles
            else:
                targets = []
                p = 0
                while mask:
                    if mask & 1:
                        targets.extend(by_part.get(p, ()))
                    mask >>= 1
                    p += 1
            for h in targets:
                lst = per.get(id(h))
                if lst is None:
                    per[id(h)] = lst = (h, [])
                lst[1].append(line)
        for h, ls in per.values():
            self._send(h, {"t": "w", "k": kind, "l": ls})
            self.stats["lines_out"] += len(ls)

    def dump_trace(self) -> None:
        """Write the relay trace (kind, namespace, name, wall-clock ns per relayed line) under NCC_TRACE_STAGES."""
        d = os.environ.get("NCC_TRACE_STAGES")
        if not d or self.trace is None:
            return
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, f"relay-{os.getpid()}.tsv"), "w") as f:
            for kind, ns, name, t in self.trace:
                f.write(f"{kind}\t{ns}/{name}\t{t}\n")

    def _send_all(self, handles: list, msg: dict) -> None:
        """One encoding of `msg` for every executor it goes to."""
        packed = msgpack.packb(msg, use_bin_type=True)
        for h in handles:
            ch = h.channel
            if ch is not None:
                ch.send_packed(packed)
                self.stats["frames"] += 1

    def _send(self, handle, msg: dict) -> None:
        ch = handle.channel
        if ch is not None:
            ch.send(msg)
            self.stats["frames"] += 1
