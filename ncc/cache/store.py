"""Thread-confined object store with secondary indices and a write-through mutation overlay.

The client-go analogues are `cache.Indexer` (thread-safe store + indices) and
`cache.MutationCache` (`NewIntegerResourceVersionMutationCache`).  The reference reads all
state through listers backed by this kind of store (controller.go:107-121), so reconciles
issue zero GETs.

The mutation overlay (`assume`) lets a reconcile see its own successful writes before the
watch event for them arrives: a subsequent reconcile of the same key then neither re-creates
an object it just created (→ 409 AlreadyExists) nor updates from a stale resourceVersion
(→ 409 Conflict).  An assumed object is shadowed as soon as the informer stores a version at
least as new, or after `assume_ttl` seconds.
"""
from __future__ import annotations

import time
from typing import Callable, Iterable

from ..api.objects import ObjectKey, key_of, rv_int

IndexFunc = Callable[[dict], Iterable[str]]


class Store:
    def __init__(self, transform: Callable[[dict], dict] | None = None, assume_ttl: float = 60.0):
        self._items: dict[ObjectKey, dict] = {}
        self._indexers: dict[str, IndexFunc] = {}
        self._indices: dict[str, dict[str, set]] = {}
        self._index_vals: dict[str, dict[ObjectKey, tuple]] = {}  # indexer → key → its current values
        self._assumed: dict[ObjectKey, tuple[dict, int, float]] = {}
        self._tombstones: dict[ObjectKey, int] = {}  # key -> RV of the observed delete
        self.transform = transform
        self.assume_ttl = assume_ttl
        # index_guard(obj): a cheap projection of everything the indexers read; an update that leaves it
        # equal skips the indexers altogether (templates: the mapped environment, i.e. the references)
        self.index_guard: Callable[[dict], object] | None = None
        # index_same(old, new): index_guard(old) == index_guard(new) in one call (a native twin); TypeError from it
        # falls back to comparing the guards
        self.index_same: Callable[[dict, dict], bool] | None = None

    # ------------------------------------------------------------ indices
    def add_indexer(self, name: str, fn: IndexFunc) -> None:
        self._indexers[name] = fn
        idx: dict[str, set] = {}
        vals: dict[ObjectKey, tuple] = {}
        for k, o in self._items.items():
            vs = tuple(fn(o))
            if vs:
                vals[k] = vs
            for v in vs:
                idx.setdefault(v, set()).add(k)
        self._indices[name] = idx
        self._index_vals[name] = vals

    def _index(self, key: ObjectKey, old: dict | None, new: dict | None) -> None:
        """Move `key` between index buckets.  Each key's current index values are remembered, so an update
        that leaves them unchanged (the common case: a spec edit keeps the references) touches no set."""
        g = self.index_guard
        if g is not None and old is not None and new is not None:
            same = self.index_same
            if same is not None:
                try:
                    if same(old, new):
                        return
                except TypeError:
                    if g(old) == g(new):
                        return
            elif g(old) == g(new):
                return
        for name, fn in self._indexers.items():
            vals = self._index_vals[name]
            ov = vals.get(key, ())
            nv = tuple(fn(new)) if new is not None else ()
            if ov == nv:
                continue
            idx = self._indices[name]
            for v in ov:
                s = idx.get(v)
                if s is not None:
                    s.discard(key)
                    if not s:
                        del idx[v]
            for v in nv:
                idx.setdefault(v, set()).add(key)
            if nv:
                vals[key] = nv
            else:
                vals.pop(key, None)

    def by_index(self, name: str, value: str) -> list[dict]:
        return [self._items[k] for k in self._indices.get(name, {}).get(value, ()) if k in self._items]

    # ------------------------------------------------------------ mutation
    def upsert(self, obj: dict) -> tuple[dict, dict | None]:
        """Store `obj` (after transform); return (stored, previous)."""
        if self.transform is not None:
            obj = self.transform(obj)
        key = key_of(obj)
        old = self._items.get(key)
        self._items[key] = obj
        if self._indexers:
            self._index(key, old, obj)
        return obj, old

    def delete(self, obj_or_key) -> dict | None:
        key = obj_or_key if isinstance(obj_or_key, tuple) else key_of(obj_or_key)
        old = self._items.pop(key, None)
        rv = -1 if isinstance(obj_or_key, tuple) else \
            rv_int((obj_or_key.get("metadata") or {}).get("resourceVersion"))
        a = self._assumed.get(key)
        if a is not None and not (rv >= 0 and a[1] > rv):
            del self._assumed[key]  # an overlay newer than the deleted version (we re-created it) survives
        if not isinstance(obj_or_key, tuple):
            if rv >= 0:
                if len(self._tombstones) > 16384:
                    self._tombstones.clear()
                self._tombstones[key] = rv
        if old is not None and self._indexers:
            self._index(key, old, None)
        return old

    def replace(self, objs: Iterable[dict], transformed: bool = False) -> tuple[list, list, list]:
        """Swap the whole content (relist).  Returns (added, updated[(old,new)], deleted).  `transformed`: the
        objects are already in stored form."""
        new_items: dict[ObjectKey, dict] = {}
        transform = None if transformed else self.transform
        old_items = self._items
        for o in objs:
            if transform is not None:
                o = transform(o)
            k = key_of(o)
            prev = old_items.get(k)
            # the cached version when the listing has the same one: a relist of an unchanged cluster then holds
            # one copy of its objects, not two, and handlers see the very same object (old is new)
            if prev is not None and (prev.get("metadata") or {}).get("resourceVersion") == \
                    (o.get("metadata") or {}).get("resourceVersion"):
                o = prev
            new_items[k] = o
        added, updated, deleted = [], [], []
        for k, o in new_items.items():
            prev = old_items.get(k)
            if prev is None:
                added.append(o)
            else:
                updated.append((prev, o))
        for k, o in old_items.items():
            if k not in new_items:
                deleted.append(o)
        self._items = new_items
        if self._assumed:  # a relist is authoritative: drop overlays for vanished or caught-up keys
            for k in list(self._assumed):
                cur = new_items.get(k)
                if cur is None or rv_int((cur.get("metadata") or {}).get("resourceVersion")) >= self._assumed[k][1]:
                    del self._assumed[k]
        for name, fn in self._indexers.items():
            idx: dict[str, set] = {}
            vals: dict[ObjectKey, tuple] = {}
            for k, o in new_items.items():
                vs = tuple(fn(o))
                if vs:
                    vals[k] = vs
                for v in vs:
                    idx.setdefault(v, set()).add(k)
            self._indices[name] = idx
            self._index_vals[name] = vals
        return added, updated, deleted

    def assume(self, obj: dict, transformed: bool = False) -> None:
        """Record a write result we made; visible to `get` until the informer catches up.
        `transformed=True`: `obj` is already in stored form (e.g. a slim object built by the writer)."""
        if self.transform is not None and not transformed:
            obj = self.transform(obj)
        key = key_of(obj)
        rv = rv_int((obj.get("metadata") or {}).get("resourceVersion"))
        if rv < 0:
            return
        cur = self._items.get(key)
        if cur is not None and rv_int((cur.get("metadata") or {}).get("resourceVersion")) >= rv:
            return
        if cur is None and self._tombstones.get(key, -1) >= rv:
            return  # a late write result for an object we have already seen deleted
        prev = self._assumed.get(key)
        if prev is not None and prev[1] >= rv:
            return
        self._assumed[key] = (obj, rv, time.monotonic() + self.assume_ttl)

    def confirm(self, key: ObjectKey, resource_version: str) -> dict | None:
        """The watch delivered exactly the version we assumed: promote it without decoding the event."""
        a = self._assumed.get(key)
        if a is None or a[1] != rv_int(resource_version):
            return None
        del self._assumed[key]
        obj = a[0]
        old = self._items.get(key)
        self._items[key] = obj
        if self._indexers:
            self._index(key, old, obj)
        return obj

    def promote(self, key, resource_version: str) -> dict | None:
        """A watch event at `resource_version` carries nothing the stored form keeps that differs from our
        assumed write result (a metadata-only store: same owners): make the overlay the stored version when the
        event is at least as new.  Without this, an echo skipped as "owners unchanged" would leave the
        pre-write version in the store once the overlay expires (`assume_ttl`), and the next relist would see
        every adopted dependent as changed."""
        a = self._assumed.get(key)
        if a is None or rv_int(resource_version) < a[1]:
            return None
        del self._assumed[key]
        obj = a[0]
        old = self._items.get(key)
        self._items[key] = obj
        if self._indexers:
            self._index(key, old, obj)
        return obj

    # ------------------------------------------------------------ reads
    def get(self, namespace: str, name: str) -> dict | None:
        key = (namespace, name)  # hashes and compares equal to ObjectKey(namespace, name), built faster
        cur = self._items.get(key)
        if self._assumed:
            a = self._assumed.get(key)
            if a is not None:
                if (cur is not None and rv_int((cur.get("metadata") or {}).get("resourceVersion")) >= a[1]) \
                        or time.monotonic() > a[2]:
                    del self._assumed[key]
                else:
                    return a[0]
        return cur

    def get_key(self, key: ObjectKey) -> dict | None:
        return self.get(key.namespace, key.name)

    def list(self, namespace: str | None = None) -> list[dict]:
        if namespace is None:
            return list(self._items.values())
        return [o for k, o in self._items.items() if k.namespace == namespace]

    def keys(self) -> list[ObjectKey]:
        return list(self._items.keys())

    def __len__(self) -> int:
        return len(self._items)

    def __contains__(self, key: ObjectKey) -> bool:
        return key in self._items
