"""In-memory versioned object store with watch fan-out and ownerRef garbage collection.

This is the state machine behind both the HTTP fake kube-apiserver (`ncc.fakeapi.server`)
and the in-process recording client (`ncc.testing.fake_client`).  It stands in for the
envtest/kind clusters the reference's CI provisions (.github/workflows/build.yaml:44-66)
and implements the apiserver behaviours the controller depends on:

* monotonically increasing integer resourceVersions (one counter per cluster, like etcd);
* list + watch from a resourceVersion with replay from a bounded history and
  `410 Gone` once the requested version has been compacted away;
* status subresource isolation (main-resource writes ignore `.status`, `/status` writes
  touch only `.status`) and no-op updates that neither bump the RV nor emit events;
* optimistic concurrency (`409 Conflict` on a stale `metadata.resourceVersion`);
* `AlreadyExists` on create, UID/creationTimestamp/generation management;
* background-style garbage collection: deleting an owner deletes dependents whose owners
  are all gone and strips dangling references from dependents that keep a live owner.

`simple=True` switches to client-go `fake.NewSimpleClientset` semantics used by the parity
tests (no UIDs, no RVs, no conflict checks, no GC, status stored verbatim) so recorded
request objects match the reference's expected actions (controller_test.go:383-466).
"""
from __future__ import annotations

import asyncio
import base64
import json
import uuid
from collections import deque
from typing import Callable

from ..api import resources as R
from ..api import selectors
from ..api.jsonenc import dumps_bytes
from ..api.objects import deep_copy, now_rfc3339
from ..api.patch import apply_patch, json_patch, merge_patch, strategic_merge_patch

_APPLY_ALWAYS = frozenset(("apiVersion", "kind", "metadata"))  # never removed by an apply that omits them
from ..api.resources import ResourceType
from ..kube import errors as E
from ..kube.client import PATCH_APPLY, PATCH_JSON, PATCH_MERGE, PATCH_STRATEGIC
from .admission import Admission

RtKey = tuple  # (group, plural)


class EventRecord:
    __slots__ = ("rv", "rt_key", "namespace", "type", "obj", "_line", "_body")

    def __init__(self, rv: int, rt_key: RtKey, namespace: str, type_: str, obj: dict):
        self.rv, self.rt_key, self.namespace, self.type, self.obj = rv, rt_key, namespace, type_, obj
        self._line = None
        self._body = None

    def body(self) -> bytes:
        """The object's JSON, encoded once for the write response and every watch line."""
        if self._body is None:
            self._body = dumps_bytes(self.obj)
        return self._body

    def line(self) -> bytes:
        """Serialised watch-stream line, computed once and shared by every watcher."""
        if self._line is None:
            self._line = b'{"type":"' + self.type.encode() + b'","object":' + self.body() + b"}\n"
        return self._line


class Mailbox:
    """Minimal single-consumer queue (the subset of asyncio.Queue a watch stream uses).  `put_nowait` is a
    deque append plus, only when the consumer is parked, one future completion — it runs once per event
    per watcher, so it must stay much cheaper than asyncio.Queue's bookkeeping."""
    __slots__ = ("_items", "_waiter")

    def __init__(self):
        self._items: deque = deque()
        self._waiter: asyncio.Future | None = None

    def put_nowait(self, item) -> None:
        self._items.append(item)
        w = self._waiter
        if w is not None:
            self._waiter = None
            if not w.done():
                w.set_result(None)

    def empty(self) -> bool:
        return not self._items

    def qsize(self) -> int:
        return len(self._items)

    def get_nowait(self):
        if not self._items:
            raise asyncio.QueueEmpty
        return self._items.popleft()

    async def get(self):
        while not self._items:
            fut = self._waiter = asyncio.get_running_loop().create_future()
            try:
                await fut
            finally:
                if self._waiter is fut:
                    self._waiter = None
        return self._items.popleft()


class Watcher:
    def __init__(self, state: "ClusterState", rt_key: RtKey, namespace: str | None, selector: str | None):
        self.state = state
        self.rt_key = rt_key
        self.namespace = namespace or None
        self.match_labels = selectors.parse(selector)
        self.everything = not selector  # no label selector: only the namespace decides
        self.queue = Mailbox()
        self.closed = False

    def wants(self, rec: EventRecord) -> bool:
        if rec.rt_key != self.rt_key:
            return False
        if self.namespace and rec.namespace != self.namespace:
            return False
        return self.match_labels((rec.obj.get("metadata") or {}).get("labels") or {})

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            self.state._watchers.discard(self)
            self.state._by_rt.get(self.rt_key, set()).discard(self)
            self.queue.put_nowait(None)


def _conflict(rt: ResourceType, name: str) -> E.Conflict:
    gr = f"{rt.plural}.{rt.group}" if rt.group else rt.plural
    return E.Conflict(f'Operation cannot be fulfilled on {gr} "{name}": the object has been modified; '
                      f"please apply your changes to the latest version and try again",
                      details={"name": name, "kind": rt.plural, "group": rt.group})


def _not_found(rt: ResourceType, name: str) -> E.NotFound:
    gr = f"{rt.plural}.{rt.group}" if rt.group else rt.plural
    return E.NotFound(f'{gr} "{name}" not found', details={"name": name, "kind": rt.plural, "group": rt.group})


def _content(obj: dict) -> dict:
    """Everything except metadata and status — the part whose change bumps `generation`."""
    return {k: v for k, v in obj.items() if k not in ("metadata", "status", "apiVersion", "kind")}


class ClusterState:
    def __init__(self, name: str = "cluster", *, simple: bool = False, history: int = 100_000,
                 status_subresource: bool = True):
        self.name = name
        self.simple = simple
        self.status_subresource = status_subresource and not simple
        self.rv = 0
        self._objects: dict[RtKey, dict[str, dict[str, dict]]] = {}
        self._types: dict[RtKey, ResourceType] = {(rt.group, rt.plural): rt for rt in R.BUILTIN}
        self._history: deque[EventRecord] = deque(maxlen=max(history, 1))
        self._watchers: set[Watcher] = set()
        self._by_rt: dict[RtKey, set] = {}  # watchers per resource type (emit only scans those)
        self._uids: dict[str, tuple] = {}  # uid -> (rt_key, ns, name)
        self._dependents: dict[str, set] = {}  # owner uid -> {(rt_key, ns, name)}
        self.write_hooks: list[Callable[[str, ResourceType, dict], None]] = []
        self.crds: dict = {}  # (group, plural) -> CRD: writes of those kinds are schema-validated (422)
        self.admission = Admission()  # server-side mutation of write bodies (defaulting/pruning, webhooks)
        self.last_record: EventRecord | None = None  # lets the HTTP layer reuse the event's encoding
        # server-side apply: the top-level fields, labels, annotations and ownerReferences (by uid) each field
        # manager applied last time, per object uid.  What a manager applied before and omits now is removed,
        # as a real apiserver does from managedFields — without this a dropped ConfigMap.binaryData would stay
        # on the object for ever.  ownerReferences is a list-map keyed by uid: an entry another manager also
        # applies stays (it is co-owned)
        self._applied: dict[str, dict[str, tuple]] = {}
        self.stats = {"create": 0, "update": 0, "status": 0, "delete": 0, "patch": 0, "get": 0, "list": 0,
                      "watch": 0, "conflict": 0, "noop_update": 0, "gc_delete": 0}

    # ------------------------------------------------------------------ registry
    def register(self, rt: ResourceType) -> None:
        self._types[(rt.group, rt.plural)] = rt

    def resource(self, group: str, plural: str) -> ResourceType:
        rt = self._types.get((group, plural))
        if rt is None:
            raise E.NotFound(f"the server could not find the requested resource ({plural}.{group})")
        return rt

    def _bucket(self, rt: ResourceType, ns: str) -> dict[str, dict]:
        by_ns = self._objects.setdefault((rt.group, rt.plural), {})
        b = by_ns.get(ns)
        if b is None:
            b = by_ns[ns] = {}
        return b

    # ------------------------------------------------------------------ events
    def _next_rv(self) -> int:
        self.rv += 1
        return self.rv

    def _validate(self, rt: ResourceType, obj: dict) -> None:
        """Structural-schema validation of a custom resource write, as the apiserver does (422 Invalid)."""
        crd = self.crds.get((rt.group, rt.plural))
        if crd is None:
            return
        from ..api.schema import validate_object
        errs = validate_object(crd, obj, rt.version)
        if errs:
            name = (obj.get("metadata") or {}).get("name", "")
            raise E.Invalid(f'{rt.kind}.{rt.group} "{name}" is invalid: [{", ".join(errs)}]',
                            details={"name": name, "group": rt.group, "kind": rt.kind,
                                     "causes": [{"message": e} for e in errs]})

    def _emit(self, rv: int, rt: ResourceType, ns: str, type_: str, obj: dict) -> None:
        rec = EventRecord(rv, (rt.group, rt.plural), ns, type_, obj)
        self.last_record = rec
        if not self.simple:
            self._history.append(rec)
        ws = self._by_rt.get(rec.rt_key)
        if ws:
            for w in tuple(ws):
                if w.everything and (not w.namespace or w.namespace == ns):
                    w.queue.put_nowait(rec)
                elif w.wants(rec):
                    w.queue.put_nowait(rec)
        for hook in self.write_hooks:
            hook(type_, rt, obj)

    # ------------------------------------------------------------------ owner index
    def _index_owners(self, rt: ResourceType, obj: dict, add: bool) -> None:
        if self.simple:
            return
        m = obj.get("metadata") or {}
        ref = ((rt.group, rt.plural), m.get("namespace", "") or "", m.get("name", ""))
        for o in m.get("ownerReferences") or ():
            u = o.get("uid")
            if not u:
                continue
            if add:
                self._dependents.setdefault(u, set()).add(ref)
            else:
                s = self._dependents.get(u)
                if s is not None:
                    s.discard(ref)
                    if not s:
                        del self._dependents[u]

    # ------------------------------------------------------------------ reads
    def get(self, rt: ResourceType, ns: str, name: str) -> dict:
        self.stats["get"] += 1
        obj = self._bucket(rt, ns if rt.namespaced else "").get(name)
        if obj is None:
            raise _not_found(rt, name)
        return obj

    def try_get(self, rt: ResourceType, ns: str, name: str) -> dict | None:
        """The stored object, or None (tests; not counted as a request)."""
        return self._bucket(rt, ns if rt.namespaced else "").get(name)

    def list(self, rt: ResourceType, ns: str | None, *, label_selector: str | None = None,
             limit: int | None = None, continue_token: str | None = None) -> dict:
        self.stats["list"] += 1
        match = selectors.parse(label_selector)
        by_ns = self._objects.get((rt.group, rt.plural), {})
        if ns and rt.namespaced:
            buckets = [(ns, by_ns.get(ns, {}))]
        else:
            buckets = sorted(by_ns.items())
        start_after = None
        list_rv = self.rv
        if continue_token:
            try:
                tok = json.loads(base64.urlsafe_b64decode(continue_token.encode()).decode())
                start_after, list_rv = tuple(tok["k"]), int(tok["rv"])
            except Exception as e:  # noqa: BLE001
                raise E.BadRequest(f"invalid continue token: {e}")
        items = []
        next_tok = None
        for bns, b in buckets:
            for nm in sorted(b):
                if start_after is not None and (bns, nm) <= start_after:
                    continue
                o = b[nm]
                if label_selector and not match((o.get("metadata") or {}).get("labels") or {}):
                    continue
                if limit and len(items) >= limit:
                    last = items[-1]["metadata"]
                    next_tok = base64.urlsafe_b64encode(json.dumps(
                        {"k": [last.get("namespace", ""), last["name"]], "rv": list_rv}).encode()).decode()
                    break
                items.append(o)
            if next_tok:
                break
        lmeta = {"resourceVersion": str(list_rv)}
        if next_tok:
            lmeta["continue"] = next_tok
        return {"apiVersion": rt.api_version, "kind": rt.list_kind, "metadata": lmeta, "items": items}

    # ------------------------------------------------------------------ writes
    def encoded(self, obj: dict) -> bytes | None:
        """JSON of `obj` if it is the object of the latest write event (already encoded once)."""
        rec = self.last_record
        return rec.body() if rec is not None and rec.obj is obj else None

    def create(self, rt: ResourceType, ns: str, obj: dict, *, owned: bool = False) -> dict:
        """`owned=True`: the caller hands over `obj` (e.g. freshly decoded from a request) — no copy."""
        if not owned:
            obj = deep_copy(obj)
        m = obj.setdefault("metadata", {})
        ns = ns if rt.namespaced else ""
        if rt.namespaced:
            if m.get("namespace") and ns and m["namespace"] != ns:
                raise E.BadRequest("the namespace of the provided object does not match the namespace sent on the request")
            m["namespace"] = ns or m.get("namespace", "")
            ns = m["namespace"]
        name = m.get("name")
        if not name:
            gen = m.get("generateName")
            if not gen:
                raise E.Invalid("metadata.name: Required value: name or generateName is required")
            name = m["name"] = gen + uuid.uuid4().hex[:5]
        b = self._bucket(rt, ns)
        if name in b:
            gr = f"{rt.plural}.{rt.group}" if rt.group else rt.plural
            raise E.AlreadyExists(f'{gr} "{name}" already exists', details={"name": name, "kind": rt.plural})
        if self.admission.active:
            self.admission.admit(rt, obj, self.crds.get((rt.group, rt.plural)))
        if self.crds:
            self._validate(rt, obj)
        if not self.simple:
            if m.get("resourceVersion"):
                raise E.BadRequest("resourceVersion should not be set on objects to be created")
            m["uid"] = str(uuid.uuid4())
            m["creationTimestamp"] = now_rfc3339()
            if rt.group:  # CRDs carry metadata.generation; core Secrets/ConfigMaps do not
                m["generation"] = 1
            m["resourceVersion"] = str(self._next_rv())
            obj["apiVersion"] = rt.api_version
            obj["kind"] = rt.kind
            if self.status_subresource and rt.has_status:
                obj.pop("status", None)
            self._uids[m["uid"]] = ((rt.group, rt.plural), ns, name)
        b[name] = obj
        self._index_owners(rt, obj, True)
        self.stats["create"] += 1
        self._emit(self.rv, rt, ns, "ADDED", obj)
        return obj

    def update(self, rt: ResourceType, ns: str, obj: dict, *, subresource: str | None = None,
               owned: bool = False) -> dict:
        ns = ns if rt.namespaced else ""
        m_in = obj.get("metadata") or {}
        name = m_in.get("name", "")
        b = self._bucket(rt, ns)
        cur = b.get(name)
        if cur is None:
            raise _not_found(rt, name)
        if self.simple:
            new = obj if owned else deep_copy(obj)
            b[name] = new
            self.stats["status" if subresource == "status" else "update"] += 1
            self._emit(self.rv, rt, ns, "MODIFIED", new)
            return new
        cm = cur["metadata"]
        rv_in = m_in.get("resourceVersion")
        if rv_in and rv_in != cm.get("resourceVersion"):
            self.stats["conflict"] += 1
            raise _conflict(rt, name)
        if subresource == "status":
            new = dict(cur)
            if "status" in obj:
                new["status"] = deep_copy(obj["status"])
            else:
                new.pop("status", None)
            new["metadata"] = dict(cm)
        else:
            new = obj if owned else deep_copy(obj)
            nm = new.setdefault("metadata", {})
            for k in ("uid", "creationTimestamp", "namespace", "name", "generation", "deletionTimestamp"):
                if k in cm:
                    nm[k] = cm[k]
                else:
                    nm.pop(k, None)
            if "managedFields" not in nm and "managedFields" in cm:
                nm["managedFields"] = cm["managedFields"]  # unset in the request: the apiserver keeps its own
            new["apiVersion"] = rt.api_version
            new["kind"] = rt.kind
            if self.status_subresource and rt.has_status:
                if "status" in cur:
                    new["status"] = cur["status"]
                else:
                    new.pop("status", None)
            if self.admission.active:
                self.admission.admit(rt, new, self.crds.get((rt.group, rt.plural)))
            if rt.group and _content(new) != _content(cur):
                nm["generation"] = int(cm.get("generation", 1)) + 1
        new["metadata"]["resourceVersion"] = cm.get("resourceVersion")
        if self.crds:
            self._validate(rt, new)
        if new == cur:
            self.stats["noop_update"] += 1
            return cur
        new["metadata"]["resourceVersion"] = str(self._next_rv())
        same_owners = (cm.get("ownerReferences") == new["metadata"].get("ownerReferences"))
        if not same_owners:
            self._index_owners(rt, cur, False)
        b[name] = new
        if not same_owners:
            self._index_owners(rt, new, True)
        self.stats["status" if subresource == "status" else "update"] += 1
        self._emit(self.rv, rt, ns, "MODIFIED", new)
        return new

    def patch(self, rt: ResourceType, ns: str, name: str, body, patch_type: str, *,
              subresource: str | None = None, manager: str = "") -> dict:
        self.stats["patch"] += 1
        ns = ns if rt.namespaced else ""
        cur = self._bucket(rt, ns).get(name)
        if patch_type == PATCH_APPLY:
            bm = body.get("metadata") or {}
            fields = (frozenset(k for k in body if k not in _APPLY_ALWAYS), frozenset(bm.get("labels") or ()),
                      frozenset(bm.get("annotations") or ()),
                      frozenset(r.get("uid") for r in bm.get("ownerReferences") or () if isinstance(r, dict)))
            if cur is None:
                body = dict(body)
                body.setdefault("metadata", {}).setdefault("name", name)
                out = self.create(rt, ns, body)
                self._applied[out["metadata"].get("uid", "")] = {manager: fields}
                return out
            new = apply_patch(cur, body)
            uid = cur["metadata"].get("uid", "")
            managers = self._applied.setdefault(uid, {})
            prev = managers.get(manager)
            if prev is not None:
                gone_refs = {r for r in prev[3] - fields[3]
                             if not any(r in f[3] for m, f in managers.items() if m != manager)}
                if gone_refs and new["metadata"].get("ownerReferences"):
                    new["metadata"] = dict(new["metadata"])
                    new["metadata"]["ownerReferences"] = [r for r in new["metadata"]["ownerReferences"]
                                                          if r.get("uid") not in gone_refs]
                for k in prev[0] - fields[0]:
                    new.pop(k, None)
                for i, mk in ((1, "labels"), (2, "annotations")):
                    gone = prev[i] - fields[i]
                    if gone and new["metadata"].get(mk):
                        kept = {k: v for k, v in new["metadata"][mk].items() if k not in gone}
                        new["metadata"] = dict(new["metadata"])
                        if kept:
                            new["metadata"][mk] = kept
                        else:
                            new["metadata"].pop(mk, None)
            managers[manager] = fields
        else:
            if cur is None:
                raise _not_found(rt, name)
            if patch_type == PATCH_JSON:
                try:
                    new = json_patch(cur, body)
                except Exception as e:  # noqa: BLE001
                    raise E.Invalid(f"json patch failed: {e}")
            elif patch_type == PATCH_STRATEGIC:
                new = strategic_merge_patch(cur, body)
            elif patch_type == PATCH_MERGE:
                new = merge_patch(cur, body)
            else:
                raise E.ApiError(f"unsupported patch type {patch_type}", code=415, reason="UnsupportedMediaType")
        new = dict(new)
        new["metadata"] = dict(new.get("metadata") or {})
        # a patch carries no precondition unless it sets one explicitly
        want_rv = ((body.get("metadata") or {}) if isinstance(body, dict) else {}).get("resourceVersion")
        new["metadata"]["resourceVersion"] = want_rv or cur["metadata"].get("resourceVersion")
        return self.update(rt, ns, new, subresource=subresource)

    def delete(self, rt: ResourceType, ns: str, name: str, *, preconditions: dict | None = None,
               propagation_policy: str | None = None) -> dict:
        ns = ns if rt.namespaced else ""
        b = self._bucket(rt, ns)
        cur = b.get(name)
        if cur is None:
            raise _not_found(rt, name)
        cm = cur.get("metadata") or {}
        if preconditions:
            if preconditions.get("uid") and preconditions["uid"] != cm.get("uid"):
                raise _conflict(rt, name)
            if preconditions.get("resourceVersion") and preconditions["resourceVersion"] != cm.get("resourceVersion"):
                raise _conflict(rt, name)
        del b[name]
        self.stats["delete"] += 1
        if self._applied:
            self._applied.pop(cm.get("uid", ""), None)
        if self.simple:
            self._emit(self.rv, rt, ns, "DELETED", cur)
            return cur
        self._index_owners(rt, cur, False)
        u = cm.get("uid")
        if u:
            self._uids.pop(u, None)
        gone = dict(cur)
        gone["metadata"] = dict(cm, resourceVersion=str(self._next_rv()))
        self._emit(self.rv, rt, ns, "DELETED", gone)
        if u:
            self._collect(u, orphan=(propagation_policy == "Orphan"))
        return gone

    def _collect(self, owner_uid: str, orphan: bool = False) -> None:
        """Garbage-collect dependents of a deleted owner (K8s GC `attemptToDeleteItem`)."""
        deps = self._dependents.pop(owner_uid, set())
        for rt_key, ns, nm in sorted(deps):
            rt = self._types[rt_key]
            obj = self._bucket(rt, ns).get(nm)
            if obj is None:
                continue
            refs = (obj.get("metadata") or {}).get("ownerReferences") or []
            solid = [r for r in refs if r.get("uid") in self._uids]
            if solid and not orphan:
                self.update(rt, ns, _with_refs(obj, solid))
            elif orphan:
                self.update(rt, ns, _with_refs(obj, [r for r in refs if r.get("uid") != owner_uid]))
            else:
                self.stats["gc_delete"] += 1
                self.delete(rt, ns, nm)

    # ------------------------------------------------------------------ watch
    def watch(self, rt: ResourceType, ns: str | None, resource_version: str | None,
              label_selector: str | None = None) -> Watcher:
        self.stats["watch"] += 1
        w = Watcher(self, (rt.group, rt.plural), ns if rt.namespaced else None, label_selector)
        if resource_version in (None, "", "0"):
            for obj in self.list(rt, ns, label_selector=label_selector)["items"]:
                w.queue.put_nowait(EventRecord(self.rv, w.rt_key, (obj.get("metadata") or {}).get("namespace", ""),
                                               "ADDED", obj))
        else:
            try:
                since = int(resource_version)
            except ValueError:
                raise E.BadRequest(f"invalid resourceVersion {resource_version!r}")
            if since < self.rv:
                if not self._history or self._history[0].rv > since + 1:
                    raise E.Gone(f"too old resource version: {since} ({self._history[0].rv - 1 if self._history else self.rv})")
                for rec in self._history:
                    if rec.rv > since and w.wants(rec):
                        w.queue.put_nowait(rec)
        self._watchers.add(w)
        self._by_rt.setdefault(w.rt_key, set()).add(w)
        return w

    def compact(self, advance: bool = False) -> None:
        """Drop all watch history (forces 410 Gone on every resume), like an etcd compaction.

        `advance`: also move the revision past every client's last-seen one (a real apiserver's revision
        keeps moving with Lease and Event writes), so that even a watcher that was fully caught up must relist
        — the relist storm of bench/suite.py config 4."""
        if advance:
            self.rv += 1
        self._history.clear()

    def close_watchers(self) -> None:
        for w in tuple(self._watchers):
            w.close()

    def count(self, rt: ResourceType, ns: str | None = None) -> int:
        by_ns = self._objects.get((rt.group, rt.plural), {})
        if ns:
            return len(by_ns.get(ns, {}))
        return sum(len(b) for b in by_ns.values())


def _with_refs(obj: dict, refs: list) -> dict:
    o = dict(obj)
    o["metadata"] = dict(obj.get("metadata") or {}, ownerReferences=refs)
    if not refs:
        o["metadata"].pop("ownerReferences")
    return o
