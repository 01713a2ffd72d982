"""The controller: informer event handlers, the work queue, and the worker pool.

Reference: `Controller` / `NewController` / `Run` / `processNextWorkItem` / `enqueueResource` /
`handleObject` in controller.go:98-426,851-884.  Queue elements are the strings
`"<kind>/<namespace>/<name>"` with kind ∈ {template, workgroup} — the reference's
`Element{objRef, objTypeName}` (controller.go:88-96) in a form the native C++ queue can hash.

Handler wiring (controller.go:286-355):
  template/workgroup  add/update → enqueue; delete → `handle_object`
  secret/configmap    add → handle_object; update → handle_object if the RV changed; delete → handle_object
`handle_object` unwraps tombstones; a deleted template is removed from every shard (compat:
inline, sequential, first error aborts; native: queued and retried); any other object
enqueues the NexusAlgorithmTemplates named in its ownerRefs that exist in the lister.
"""
from __future__ import annotations

import asyncio
import contextvars
import logging
import os
import time

import msgpack

from .. import native as _native
from ..api import constants as C
from ..api.objects import ObjectKey, meta
from ..api.refs import configmap_names, same_references, secret_names, template_owner_names
from ..cache.informer import DeletedFinalStateUnknown, Informer
from ..telemetry.statsd import Metrics, NullMetrics
from ..workqueue.queue import WorkQueue
from .events import EventRecorder, FakeRecorder
from .executor import key_part
from .options import ControllerOptions
from .reports import make_report_table
from .reconcile import ReconcileMixin, spec_matches, data_matches

log = logging.getLogger("ncc.controller")

_pass_state: contextvars.ContextVar = contextvars.ContextVar("ncc_pass_state", default=None)


def make_key(kind: str, namespace: str, name: str) -> str:
    return f"{kind}/{namespace}/{name}"


def split_key(key: str) -> tuple[str, str, str]:
    kind, ns, name = key.split("/", 2)
    return kind, ns, name


def _reference_guard(t: dict):
    """What the template indices read: the namespace and the mapped environment — of a slim template, the
    digest of the environment's text (an int compare instead of a list-of-dicts compare)."""
    spec = t.get("spec") or {}
    r = spec.get("_rfp")
    if r is None:
        r = (spec.get("runtimeEnvironment") or {}).get("mappedEnvironmentVariables")
    return (t.get("metadata") or {}).get("namespace"), r


class Controller(ReconcileMixin):
    def __init__(self, *, alias: str, namespace: str, client, shards: list,
                 template_informer: Informer, workgroup_informer: Informer,
                 secret_informer: Informer, configmap_informer: Informer,
                 options: ControllerOptions | None = None, recorder: EventRecorder | None = None,
                 metrics: Metrics | None = None, queue: WorkQueue | None = None,
                 shard_names: list[str] | None = None):
        self.alias = alias
        self.namespace = namespace
        self.client = client
        self.shards = list(shards)
        self.options = options or ControllerOptions.compat()
        self.recorder = recorder or FakeRecorder(keep=False)
        self.metrics = metrics or NullMetrics()
        self.template_informer = template_informer
        self.workgroup_informer = workgroup_informer
        self.secret_informer = secret_informer
        self.configmap_informer = configmap_informer
        self.template_lister = template_informer.lister
        self.workgroup_lister = workgroup_informer.lister
        self.secret_lister = secret_informer.lister
        self.configmap_lister = configmap_informer.lister
        o = self.options
        self.queue = queue or WorkQueue(base_delay=o.failure_base_delay, max_delay=o.failure_max_delay,
                                        qps=o.rate_limit_qps, burst=o.rate_limit_burst, native=o.native_queue)
        self._pending_deletes: set = set()
        self._pending_workgroup_deletes: set = set()
        self._last_event = float("-inf")  # monotonic time of the last event-driven enqueue (coalescing)
        self._run_len = 0  # events in the current run (coalescing)
        self._workers: list[asyncio.Task] = []
        self._aux: list[asyncio.Task] = []
        self.stats = {"reconciles": 0, "errors": 0, "template": 0, "workgroup": 0, "reports": 0,
                      "reports_pending": 0, "early_passes_skipped": 0, "inline_finishes": 0, "inline_superseded": 0}
        self._inline_keys: set = set()  # coordinator: keys with a complete report set, finished in one batch
        # key -> (template object, shard-name list) whose status finish_inline found final (identity memo)
        self._inline_status_ok: dict = {}
        self._inline_timer = None
        self.ready = asyncio.Event()  # workers running
        self.caches_synced = asyncio.Event()  # controller (and shard) caches synced
        self.role = o.role
        # coordinator role: key -> {shard: (uid, generation, error)} of the executors' reports (native table)
        self.reports = make_report_table()
        # parent of partitioned coordinators: callable(partition, [raw report message, ...]) relaying the
        # reports on other partitions' keys (the report table sets them aside)
        self.forward_reports = None
        self.all_shard_names = list(shard_names) if shard_names is not None else [s.name for s in self.shards]
        self.reporter = None  # executor role: callable(msg) sending results to the coordinator
        # executor role with the watch relay: callable(kind index, "ns/name") asking the coordinator for a
        # controller object this executor has not received (see `_executor_fetch_reference`)
        self.need = None
        self.on_ready = None  # executor role: called once caches are synced and workers run
        self.on_synced = None  # executor role: called once caches are synced (before a gate opens)
        self._pending_event: set = set()
        # coordinator: template key -> {shard: signature of the failure whose Warning Events were recorded}
        self._failure_events: dict[str, dict] = {}
        # adoption_cache: template key → resourceVersion whose references were last verified as adopted
        self._adopted: dict[str, str] = {}
        if o.assume_writes:
            for inf in (template_informer, workgroup_informer, secret_informer, configmap_informer):
                inf.echo_fastpath = True
        if o.mode == "native":
            # reverse index template ← referenced Secret/ConfigMap, so dependents map to templates even
            # before adoption has stamped ownerRefs on them
            self.template_informer.store.add_indexer(
                "secret", lambda t: [f"{meta(t).get('namespace', '')}/{n}" for n in secret_names(t)])
            self.template_informer.store.add_indexer(
                "configmap", lambda t: [f"{meta(t).get('namespace', '')}/{n}" for n in configmap_names(t)])
            # both indices read only the namespace and the mapped environment
            self.template_informer.store.index_guard = _reference_guard
            mod = _native.load()
            if mod is not None and hasattr(mod, "template_index_same"):
                self.template_informer.store.index_same = mod.template_index_same
        self._register_handlers()

    @property
    def all_shard_names(self) -> list[str]:
        return self._all_shard_names

    @all_shard_names.setter
    def all_shard_names(self, names) -> None:
        # the report table decides completeness against this list: assign a new list, never mutate in place
        self._all_shard_names = list(names)
        self.reports.set_shards(self._all_shard_names)

    # ================================================================== handlers
    def _register_handlers(self) -> None:
        o = self.options
        self.template_informer.add_event_handler(
            on_add=lambda obj: self.enqueue_resource(obj, C.KIND_TEMPLATE),
            on_update=self._template_update_handler(),
            on_delete=self._on_template_delete)
        self.workgroup_informer.add_event_handler(
            on_add=lambda obj: self.enqueue_resource(obj, C.KIND_WORKGROUP),
            on_update=lambda old, new: self._on_crd_update(old, new, C.KIND_WORKGROUP),
            on_delete=self._on_workgroup_delete)
        for inf, idx in ((self.secret_informer, "secret"), (self.configmap_informer, "configmap")):
            inf.add_event_handler(on_add=lambda o, i=idx: self._on_dependent(o, i),
                                  on_update=lambda old, new, i=idx: self._on_dependent_update(old, new, i),
                                  on_delete=lambda o, i=idx: self._on_dependent(o, i))
        if o.watch_shards:
            for shard in self.shards:
                self._register_shard_handlers(shard)

    def _template_update_handler(self):
        """The template informer's on_update: `_on_crd_update` (the specification), or — coordinator role with the
        adoption cache, the native report table loaded — the same decision in one native call
        (`ReportTable.template_update`), falling back to `_on_crd_update` on anything of an unexpected type."""
        fn = getattr(self.reports, "template_update", None)
        if fn is None or self.role != "coordinator" or not self.options.adoption_cache:
            return lambda old, new: self._on_crd_update(old, new, C.KIND_TEMPLATE)
        gf = bool(self.options.generation_filter)

        def on_update(old, new):
            try:
                r = fn(old, new, self._adopted, gf, same_references)
            except TypeError:
                return self._on_crd_update(old, new, C.KIND_TEMPLATE)
            if r is None:
                return None
            if r is False:
                self.stats["early_passes_skipped"] += 1
                return None
            self._enqueue_key(r)
        return on_update

    def _on_crd_update(self, old: dict, new: dict, kind: str) -> None:
        o = self.options
        om, nm = old.get("metadata") or {}, new.get("metadata") or {}
        nrv = nm.get("resourceVersion")
        orv = om.get("resourceVersion")
        key = None
        if o.adoption_cache and kind == C.KIND_TEMPLATE:
            # adoption depends on the references and the dependents' ownerRefs (whose changes arrive as
            # dependent events): a new template version with the same references stays adopted
            key = f"{kind}/{nm.get('namespace') or ''}/{nm.get('name', '')}"
            adopted = self._adopted
            if adopted.get(key) == orv and om.get("uid") == nm.get("uid") and same_references(old, new):
                adopted[key] = nrv
        if o.generation_filter:
            if orv == nrv:
                return  # informer resync: nothing changed
            gen = om.get("generation")
            if gen is not None and gen == nm.get("generation") and om.get("labels") == nm.get("labels") \
                    and om.get("annotations") == nm.get("annotations") and old.get("spec") == new.get("spec"):
                return  # status-only change (typically our own status write)
        if self.role == "coordinator" and o.adoption_cache:
            # A new version of an initialised, adopted object has nothing to do here until every shard has
            # reported on it, and the last report enqueues it: skip the early pass.
            if key is None:
                key = make_key(kind, nm.get("namespace", "") or "", nm.get("name", ""))
            if (new.get("status") or {}).get("conditions") and \
                    (kind != C.KIND_TEMPLATE or self._adopted.get(key) == nrv) and \
                    self.shard_ready_ok(key, new) is None:
                self.stats["early_passes_skipped"] += 1
                return
        self._enqueue_key(key or make_key(kind, nm.get("namespace", "") or "", nm.get("name", "")))

    def _on_dependent(self, obj, index: str):
        obj = self._unwrap(obj)
        if self.options.mode == "native":
            # templates referencing the object (reverse index), then owners that no longer reference it
            # (handleObject's ownerRef walk, controller.go:206-223) — each template enqueued once
            ns, name = meta(obj).get("namespace", "") or "", meta(obj).get("name", "")
            seen = set()
            adopted = self._adopted
            for t in self.template_informer.store.by_index(index, f"{ns}/{name}"):
                tn = meta(t).get("name", "")
                seen.add(tn)
                key = make_key(C.KIND_TEMPLATE, ns, tn)
                adopted.pop(key, None)  # the dependent's ownership may have changed: re-check adoption
                self._enqueue_key(key)
            if isinstance(obj, dict) and obj.get("kind") != C.TEMPLATE_KIND:
                for ref in meta(obj).get("ownerReferences") or ():
                    if ref.get("kind") != C.TEMPLATE_KIND or ref.get("name", "") in seen:
                        continue
                    if self.template_lister.try_get(ns, ref.get("name", "")) is None:
                        return None  # the reference stops at the first orphaned owner (controller.go:215-218)
                    self._enqueue_key(make_key(C.KIND_TEMPLATE, ns, ref.get("name", "")))
                return None
        return self.handle_object(obj)

    def _on_dependent_update(self, old: dict, new: dict, index: str = "secret") -> None:
        om, nm = meta(old), meta(new)
        if om.get("resourceVersion") == nm.get("resourceVersion"):
            # Periodic resync will send update events for all known Secrets/ConfigMaps (controller.go:324-328).
            return
        if self.options.dependent_data_filter and old.get("data") == new.get("data") \
                and old.get("binaryData") == new.get("binaryData") and old.get("type") == new.get("type") \
                and template_owner_names(old) == template_owner_names(new) \
                and (not self.options.sync_dependent_metadata or
                     (om.get("labels"), om.get("annotations")) == (nm.get("labels"), nm.get("annotations"))):
            return  # e.g. our own adoption PUT: ownerRef UIDs changed, payload did not
        if self.options.role == "coordinator" and om.get("ownerReferences") == nm.get("ownerReferences"):
            return  # payload changes are the executors' business; the coordinator only adopts and reports
        self._on_dependent(new, index)

    def enqueue_resource(self, obj, kind: str) -> None:
        """enqueueResource (controller.go:136-162)."""
        if isinstance(obj, DeletedFinalStateUnknown):
            obj = obj.obj
        m = meta(obj)
        self._enqueue_key(make_key(kind, m.get("namespace", "") or "", m.get("name", "")))

    def _enqueue_key(self, key: str) -> None:
        """Event-driven enqueue; native mode coalesces bursts (a template and its Secret/ConfigMap
        changing together) into one reconcile by parking the key for `coalesce_window` seconds.  Only
        inside a burst — another event less than one window ago: an isolated change after a quiet window
        is reconciled at once and pays no coalescing delay."""
        part = self.options.partition
        if part is not None and key_part(key, part[1]) != part[0]:
            return  # another executor of this shard group owns the key
        delay = self._coalesce_delay()
        if delay > 0:
            self.queue.add_after(key, delay)
        else:
            self.queue.add(key)

    BURST_MIN = 32  # events in a run (each < one window after the previous) before coalescing starts

    def _coalesce_delay(self) -> float:
        """The coalesce window inside a burst — a run of more than BURST_MIN events, each less than one window
        after the previous, while at least BURST_MIN keys are queued, running or parked — else 0: an isolated
        change or a small batch is reconciled at once (back-to-back small batches too: a run alone is not
        load)."""
        w = self.options.coalesce_window
        if w <= 0:
            return 0.0
        now = time.monotonic()
        self._run_len = self._run_len + 1 if now - self._last_event < w else 1
        self._last_event = now
        if self._run_len <= self.BURST_MIN:
            return 0.0
        core = self.queue.core
        load = len(self._inline_keys) + core.length() + core.processing() + core.waiting()
        return w if load >= self.BURST_MIN else 0.0

    def _unwrap(self, obj):
        if isinstance(obj, DeletedFinalStateUnknown):
            log.debug("Recovered deleted object %s", obj.key)
            return obj.obj
        return obj

    def _on_template_delete(self, obj):
        obj = self._unwrap(obj)
        return self._handle_template_delete(obj)

    def _on_workgroup_delete(self, obj):
        obj = self._unwrap(obj)
        if self.options.propagate_workgroup_deletes:
            key = ObjectKey(meta(obj).get("namespace", ""), meta(obj).get("name", ""))
            self._pending_workgroup_deletes.add(tuple(key))
            self.enqueue_resource(obj, C.KIND_WORKGROUP)
            return None
        # reference: a deleted workgroup goes through handleObject's default branch (controller.go:206-223)
        return self._handle_dependent(obj)

    def handle_object(self, obj):
        """handleObject (controller.go:169-224).  Returns an awaitable for the inline template-delete path."""
        obj = self._unwrap(obj)
        if not isinstance(obj, dict):
            log.error("Error decoding object, invalid type %s", type(obj).__name__)
            return None
        if obj.get("kind") == C.TEMPLATE_KIND:
            return self._handle_template_delete(obj)
        return self._handle_dependent(obj)

    def _handle_dependent(self, obj: dict):
        ns = meta(obj).get("namespace", "") or ""
        for ref in meta(obj).get("ownerReferences") or ():
            if ref.get("kind") != C.TEMPLATE_KIND:
                continue
            template = self.template_lister.try_get(ns, ref.get("name", ""))
            if template is None:
                log.debug("Ignore orphaned object %s/%s (template %s)", ns, meta(obj).get("name"), ref.get("name"))
                return None  # the reference returns on the first orphaned owner (controller.go:215-218)
            self.enqueue_resource(template, C.KIND_TEMPLATE)
        return None

    def _handle_template_delete(self, obj: dict):
        ns, name = meta(obj).get("namespace", "") or "", meta(obj).get("name", "")
        if self.options.queued_deletes:
            self._pending_deletes.add((ns, name))
            self._enqueue_key(make_key(C.KIND_TEMPLATE, ns, name))
            return None
        return self._delete_template_inline(obj)

    async def _delete_template_inline(self, obj: dict) -> None:
        """controller.go:195-205: sequential, no retry, abort on the first failing shard."""
        for shard in self.shards:
            try:
                await shard.delete_template(obj)
            except Exception as e:  # noqa: BLE001
                log.error("Error deleting Template from a connected shard %s: %s", shard.name, e)
                return

    # ------------------------------------------------------------ shard-side drift watch (native)
    def repair_lost_owners(self, shard, index: str, obj: dict) -> None:
        """A shard Secret/ConfigMap in sync, unless a referencing template whose shard copy exists lost its
        ownerRef on it (another writer replaced the list: two creating applies at once, a user's edit): that
        template's pass puts it back — or shard GC could delete the copy with the other owners."""
        m = meta(obj)
        ns, name = m.get("namespace", ""), m.get("name", "")
        uids = {r.get("uid") for r in m.get("ownerReferences") or ()}
        for t in self.template_informer.store.by_index(index, f"{ns}/{name}"):
            tn = meta(t).get("name", "")
            st = shard.template_lister.try_get(ns, tn)
            if st is not None and meta(st).get("uid") not in uids:
                self._enqueue_key(make_key(C.KIND_TEMPLATE, ns, tn))

    def _register_shard_handlers(self, shard) -> None:
        def template_changed(old, new=None):
            obj = self._unwrap(new if new is not None else old)
            deleted = new is None
            ns, name = meta(obj).get("namespace", ""), meta(obj).get("name", "")
            ctl = self.template_lister.try_get(ns, name)
            if ctl is None:
                return
            if deleted or not spec_matches(ctl.get("spec"), obj):
                self._enqueue_key(make_key(C.KIND_TEMPLATE, ns, name))

        def workgroup_changed(old, new=None):
            obj = self._unwrap(new if new is not None else old)
            deleted = new is None
            ns, name = meta(obj).get("namespace", ""), meta(obj).get("name", "")
            ctl = self.workgroup_lister.try_get(ns, name)
            if ctl is None:
                return
            if deleted or not spec_matches(ctl.get("spec"), obj):
                self._enqueue_key(make_key(C.KIND_WORKGROUP, ns, name))

        sync_meta = self.options.sync_dependent_metadata

        def dependent_changed(lister, with_binary, index):
            def h(old, new=None):
                obj = self._unwrap(new if new is not None else old)
                deleted = new is None
                ns, name = meta(obj).get("namespace", ""), meta(obj).get("name", "")
                src = lister.try_get(ns, name)
                if src is None:
                    return
                if not deleted and data_matches(src, obj, with_binary) and \
                        (not sync_meta or shard.dependent_metadata_matches(src, obj)):
                    self.repair_lost_owners(shard, index, obj)
                    return
                for owner in template_owner_names(obj) or template_owner_names(src):
                    if self.template_lister.try_get(ns, owner) is not None:
                        self._enqueue_key(make_key(C.KIND_TEMPLATE, ns, owner))
            return h

        shard.template_informer.add_event_handler(on_update=template_changed, on_delete=template_changed)
        shard.workgroup_informer.add_event_handler(on_update=workgroup_changed, on_delete=workgroup_changed)
        shard.secret_informer.add_event_handler(on_update=dependent_changed(self.secret_lister, False, "secret"),
                                                on_delete=dependent_changed(self.secret_lister, False, "secret"))
        shard.configmap_informer.add_event_handler(
            on_update=dependent_changed(self.configmap_lister, self.options.sync_binary_data, "configmap"),
            on_delete=dependent_changed(self.configmap_lister, self.options.sync_binary_data, "configmap"))

    # ================================================================== coordinator / executor plumbing
    def _report(self, kind: str, namespace: str, name: str, obj: dict, results: dict) -> None:
        """Executor → coordinator: outcome of one pass over this executor's shards."""
        if self.reporter is None:
            return
        m = meta(obj)
        self.reporter({"t": "report", "k": make_key(kind, namespace, name), "u": m.get("uid", ""),
                       "g": int(m.get("generation") or 0), "r": results, "w": self._last_pass_wrote()})

    def on_executor_message(self, index: int, msg: dict) -> None:
        """Coordinator: fold one decoded executor message (tests, and executors without raw frames)."""
        if isinstance(msg, dict) and msg.get("t") == "report":
            self.on_executor_frame(index, msgpack.packb(msg, use_bin_type=True), False)

    def on_executor_frame(self, index: int, body: bytes, batch: bool) -> list:
        """Coordinator: fold a raw IPC frame of executor `index` into the report table and re-evaluate
        the objects whose report set it completed.  Returns the frame's other messages, decoded."""
        complete, wrote, errors, others, reports, pending = self.reports.feed(body, batch)
        self._folded(complete, wrote, errors, reports, pending)
        return others

    def on_executor_stream(self, index: int, buf, start: int) -> tuple[list, int]:
        """Coordinator: fold every complete frame of executor `index`'s byte stream from `start` (ipc.py
        framing, parsed natively).  Returns (the other messages, decoded; the offset after the last frame)."""
        complete, wrote, errors, others, reports, pending, end = self.reports.feed_stream(buf, start)
        self._folded(complete, wrote, errors, reports, pending)
        return others, end

    def _folded(self, complete: list, wrote: list, errors: list, reports: int, pending: int) -> None:
        if self.forward_reports is not None:
            for part, msgs in self.reports.take_forwards().items():
                self.forward_reports(part, msgs)
        st = self.stats
        st["reports"] += reports
        st["reports_pending"] += pending
        for shard in errors:
            self.metrics.count(C.SHARD_SYNC_ERRORS_METRIC, 1, {"shard": shard})
        if wrote:
            self._pending_event.update(wrote)
        # Only a complete set of reports for this object version can change its status: re-evaluate
        # then, instead of once per executor report (N× fewer coordinator passes at N shards).
        if not complete:
            return
        if not self.options.inline_finish:
            for key in complete:
                self._enqueue_key(key)
            return
        self._inline_keys.update(complete)  # _reports_complete for the whole batch
        if self._inline_timer is None:
            delay = self._coalesce_delay()
            loop = asyncio.get_running_loop()
            self._inline_timer = loop.call_later(delay, self._flush_inline) if delay > 0 else \
                loop.call_soon(self._flush_inline)

    def _reports_complete(self, key: str) -> None:
        if not self.options.inline_finish:
            self._enqueue_key(key)
            return
        # Complete: finish it in the next batch (coalesced like any event-driven enqueue); keys that need a
        # real pass go to the work queue from there.
        self._inline_keys.add(key)
        if self._inline_timer is None:
            delay = self._coalesce_delay()
            loop = asyncio.get_running_loop()
            self._inline_timer = loop.call_later(delay, self._flush_inline) if delay > 0 else \
                loop.call_soon(self._flush_inline)

    # keys finished per loop iteration: a wave's worth of completions must not hold up the loop (the watch
    # lines the relay forwards wait behind it); NCC_INLINE_BATCH overrides (experiments)
    INLINE_BATCH = int(os.environ.get("NCC_INLINE_BATCH", "256"))

    def _flush_inline(self) -> None:
        self._inline_timer = None
        pending = self._inline_keys
        if len(pending) > self.INLINE_BATCH:
            keys = [pending.pop() for _ in range(self.INLINE_BATCH)]
            self._inline_timer = asyncio.get_running_loop().call_soon(self._flush_inline)
        else:
            keys, self._inline_keys = pending, set()
        for key in self.finish_inline_many(keys):
            self.queue.add(key)

    def shard_ready_ok(self, key: str, obj: dict):
        """None while some shard has not reported on this object version, else whether all succeeded."""
        m = obj.get("metadata") or {}
        return self.reports.ready_ok(key, m.get("uid") or "", m.get("generation") or 0)

    def shard_readiness(self, key: str, obj: dict):
        """None while some shard has not reported on this object version, else {shard: error|None}."""
        m = obj.get("metadata") or {}
        return self.reports.readiness(key, m.get("uid", ""), int(m.get("generation") or 0))

    def debug_snapshot(self) -> dict:
        """Queue/informer/shard state for operators (SIGUSR1 dump, /debug/state)."""
        core = self.queue.core

        def inf(i: Informer) -> dict:
            return {"synced": i.has_synced(), "objects": len(i.store), "events": i.events, "relists": i.relists,
                    "last_rv": i.last_rv, "last_error": repr(i.last_error) if i.last_error else None}
        return {
            "role": self.role, "stats": dict(self.stats),
            "queue": {"depth": core.length(), "waiting": core.waiting(), "processing": core.processing(),
                      **self.queue.metrics},
            "informers": {n: inf(i) for n, i in (("templates", self.template_informer),
                                                 ("workgroups", self.workgroup_informer),
                                                 ("secrets", self.secret_informer),
                                                 ("configmaps", self.configmap_informer))},
            "shards": {s.name: {n: inf(i) for n, i in (("templates", s.template_informer),
                                                       ("workgroups", s.workgroup_informer),
                                                       ("secrets", s.secret_informer),
                                                       ("configmaps", s.configmap_informer))}
                       for s in self.shards},
            "pending_deletes": len(self._pending_deletes), "shard_state": len(self.reports),
            "failing": self.failing_by_shard(),
        }

    def failing_counts(self) -> dict:
        """Per shard served, how many templates' last sync there failed (0 for the healthy ones)."""
        counts = {s: 0 for s in self.all_shard_names}
        for per_shard in self._failure_events.values():
            for shard in per_shard:
                counts[shard] = counts.get(shard, 0) + 1
        return counts

    def failing_by_shard(self, limit: int = 100) -> dict:
        """Coordinator: the objects whose last complete report set failed, per shard — template key, failure
        class, the object the shard refused (kind/name), HTTP code and message (ncc/controller/failures.py);
        at most `limit` per shard.  The operator's per-shard view of what the Warning Events announced."""
        out: dict = {}
        for key in sorted(self._failure_events):
            for shard, (_sig, f) in sorted(self._failure_events[key].items()):
                lst = out.setdefault(shard, [])
                if len(lst) < limit:
                    lst.append({"key": key, "class": f.get("c", ""), "kind": f.get("k", ""), "name": f.get("n", ""),
                                "code": f.get("h", 0), "message": f.get("m", "")})
        return out

    # ================================================================== helpers
    def _assume(self, informer: Informer, res):
        if self.options.assume_writes and isinstance(res, dict):
            informer.store.assume(res)
        return res

    def _begin_pass(self) -> None:
        """Start write-tracking for one reconcile (children spawned by gather share the state)."""
        _pass_state.set([False])

    def _pass_wrote(self) -> None:
        st = _pass_state.get()
        if st is not None:
            st[0] = True

    def _last_pass_wrote(self) -> bool:
        st = _pass_state.get()
        return bool(st and st[0])

    # ================================================================== worker loop
    async def process_next_work_item(self) -> bool:
        """processNextWorkItem (controller.go:373-426)."""
        key = await self.queue.get()
        if key is None:
            return False
        start = time.monotonic()
        depth = len(self.queue)
        _pass_state.set([False])
        try:
            kind, ns, name = split_key(key)
            self.stats["reconciles"] += 1
            if kind == C.KIND_TEMPLATE:
                handler = self.sync_template
            elif kind == C.KIND_WORKGROUP:
                handler = self.sync_workgroup
            else:
                self.queue.forget(key)
                return True
            self.stats[kind] += 1
            try:
                await handler(ns, name)
                self.queue.forget(key)
            except asyncio.CancelledError:
                raise
            except Exception as e:  # noqa: BLE001
                self.stats["errors"] += 1
                log.info("Error syncing %s; re-queuing for later retry: %s", key, e)
                self.queue.add_rate_limited(key)
                if self.options.mode == "native":
                    self.metrics.count(C.RECONCILE_ERRORS_METRIC, 1, {"kind": kind})
        finally:
            self.metrics.gauge(C.WORKQUEUE_LENGTH_METRIC, depth)
            self.metrics.gauge_duration(C.RECONCILE_LATENCY_METRIC, start)
            self.queue.done(key)
        return True

    async def _run_worker(self) -> None:
        """wait.UntilWithContext(ctx, runWorker, 1s): restart the loop a second after a crash."""
        while True:
            try:
                while await self.process_next_work_item():
                    pass
                return
            except asyncio.CancelledError:
                raise
            except Exception:  # noqa: BLE001 — HandleCrash
                log.exception("worker crashed; restarting in 1s")
                await asyncio.sleep(1.0)

    # ------------------------------------------------------------------ shard membership (hot reload)
    def add_shard(self, shard) -> None:
        """Start serving a new shard (in-process shards; the coordinator uses `set_shard_names`)."""
        self.shards.append(shard)
        if self.options.watch_shards:
            self._register_shard_handlers(shard)
        shard.start()
        if shard.name not in self.all_shard_names:
            self.all_shard_names = self.all_shard_names + [shard.name]

    async def remove_shard(self, name: str) -> None:
        for shard in [s for s in self.shards if s.name == name]:
            self.shards.remove(shard)
            await shard.stop()
        if name in self.all_shard_names:
            self.all_shard_names = [s for s in self.all_shard_names if s != name]
        self.reports.drop_shards([name])

    def set_shard_names(self, names: list[str]) -> None:
        """Coordinator: the shard set changed; statuses are re-derived from the executors' reports."""
        gone = set(self.all_shard_names) - set(names)
        self.all_shard_names = list(names)
        if gone:
            self.reports.drop_shards(sorted(gone))

    async def wait_for_caches(self) -> bool:
        """Run's cache barrier (controller.go:862-871)."""
        ok = await asyncio.gather(*(i.wait_for_sync() for i in (self.secret_informer, self.configmap_informer,
                                                                 self.template_informer, self.workgroup_informer)))
        if not all(ok):
            return False
        log.info("Controller informers synced")
        t = self.options.wait_for_shards_timeout
        if t is None:
            for shard in self.shards:  # sequential and unbounded, like the reference
                await shard.wait_for_sync()
        else:
            res = await asyncio.gather(*(s.wait_for_sync(t) for s in self.shards))
            for s, r in zip(self.shards, res):
                if not r:
                    log.warning("shard %s did not sync within %.1fs; continuing without it for now", s.name, t)
        log.info("Shard informers synced")
        return True

    def start_workers(self, workers: int | None = None) -> None:
        n = workers or self.options.workers
        self._workers = [asyncio.ensure_future(self._run_worker()) for _ in range(n)]
        if self.options.orphan_sweep:
            self.sweep_orphans()
        if self.options.full_resync_period > 0:
            self._aux.append(asyncio.ensure_future(self._full_resync_loop()))
        self.ready.set()
        if self.on_ready is not None:
            self.on_ready()
        log.info("Started %d workers", n)

    def sweep_orphans(self) -> int:
        """Enqueue shard objects we own whose controller object no longer exists."""
        n = 0
        for shard in self.shards:
            for st in shard.template_lister.list():
                ns, name = meta(st).get("namespace", ""), meta(st).get("name", "")
                if self._is_ours(st) and self.template_lister.try_get(ns, name) is None:
                    self._enqueue_key(make_key(C.KIND_TEMPLATE, ns, name))
                    n += 1
            if self.options.propagate_workgroup_deletes:
                for sw in shard.workgroup_lister.list():
                    ns, name = meta(sw).get("namespace", ""), meta(sw).get("name", "")
                    if self._is_ours(sw) and self.workgroup_lister.try_get(ns, name) is None:
                        self._enqueue_key(make_key(C.KIND_WORKGROUP, ns, name))
                        n += 1
        return n

    def enqueue_all(self, part: tuple | None = None) -> None:
        """Every template and workgroup (only the keys of partition `part` = (p, C) when given)."""
        for lister, kind in ((self.template_lister, C.KIND_TEMPLATE), (self.workgroup_lister, C.KIND_WORKGROUP)):
            for obj in lister.list():
                m = meta(obj)
                key = make_key(kind, m.get("namespace", "") or "", m.get("name", ""))
                if part is None or key_part(key, part[1]) == part[0]:
                    self._enqueue_key(key)

    async def _full_resync_loop(self) -> None:
        while True:
            await asyncio.sleep(self.options.full_resync_period)
            self.enqueue_all()
            if self.options.orphan_sweep:
                self.sweep_orphans()

    async def run(self, stop: asyncio.Event, workers: int | None = None, gate: asyncio.Event | None = None) -> None:
        """Run (controller.go:851-884): cache barrier, workers, block until `stop`.

        With `gate` (a warm standby under leader election, or an executor pre-spawned for one) the caches
        sync and keys queue up as usual, but the workers start only once the gate opens."""
        log.info("Starting NexusAlgorithmTemplate controller")
        log.info("Waiting for informer caches to sync")
        sync = asyncio.ensure_future(self.wait_for_caches())
        if not await self._until(sync, stop):
            return
        if not sync.result():
            raise RuntimeError("failed to wait for caches to sync")
        self.caches_synced.set()
        if self.on_synced is not None:
            self.on_synced()
        if gate is not None and not gate.is_set():
            log.info("Caches synced; standing by until this replica leads")
            if not await self._until(asyncio.ensure_future(gate.wait()), stop):
                return
        self.start_workers(workers)
        await stop.wait()
        log.info("Shutting down workers")
        await self.shutdown()

    async def _until(self, fut: asyncio.Future, stop: asyncio.Event) -> bool:
        """Wait for `fut` unless `stop` comes first (then shut down and return False)."""
        stopper = asyncio.ensure_future(stop.wait())
        done, _ = await asyncio.wait({fut, stopper}, return_when=asyncio.FIRST_COMPLETED)
        if fut not in done:
            fut.cancel()
            await self.shutdown()
            return False
        stopper.cancel()
        return True

    def abort_workers(self) -> None:
        """Leadership lost: cancel every worker now — a reconcile must not keep writing while another
        replica may already hold the Lease."""
        self.queue.shutdown()
        for t in self._workers + self._aux:
            t.cancel()

    async def shutdown(self) -> None:
        self.queue.shutdown()
        for t in self._aux:
            t.cancel()
        if self._workers:
            _, pending = await asyncio.wait(self._workers, timeout=5.0)
            for t in pending:
                t.cancel()
        self._workers = []
        self._aux = []
