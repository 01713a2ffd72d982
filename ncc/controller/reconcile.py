"""Reconcilers: template fan-out, workgroup fan-out, adoption, status conditions, ownership.

Reference-compat semantics follow controller.go line by line in *behaviour* (ordering of API
writes, error/event emission, fail-fast), which the parity tests pin against the reference's
expected action lists (controller_test.go:800-1285).  Native semantics (selected by
`ControllerOptions`) change scheduling, not outcomes: shards are reconciled concurrently with
per-shard failure isolation, dependents within a shard are written concurrently after the
template exists (the template UID is needed for their ownerRefs), write races
are resolved by refetching, and data+owner changes go out as a single PUT.

Citations: template sync controller.go:761-845; workgroup sync :697-756; adoption :647-695;
dependents :504-626; ownership :482-502; status :428-480; shard names :628-635.
"""
from __future__ import annotations

import asyncio
import logging
import time

from ..api import constants as C
from ..api import resources as R
from ..api.constants import go_quote as q
from ..api.fingerprint import SLIM_FP, SLIM_STATUS_FP, SLIM_WROTE, fingerprint
from ..api.objects import meta, normalize_data, now_rfc3339, with_fields
from ..api.refs import (configmap_names, dependent_names, is_owned_by_uid, ready_condition, same_references,
                        secret_names, template_owner_ref)
from ..kube import errors as E
from ..kube.client import PATCH_MERGE, PATCH_STRATEGIC
from . import failures as F

log = logging.getLogger("ncc.reconcile")
_SYNCED_MESSAGE = C.MESSAGE_RESOURCE_SYNCED.format(C.TEMPLATE_KIND)


def _write_target(op: str, args: tuple) -> tuple:
    """(namespace, name) of the object a Shard write op touches, from its positional arguments."""
    if op in ("create_secret", "create_configmap"):  # (shard_template, src, fm): src's name, template's ns
        return meta(args[0]).get("namespace", ""), meta(args[1]).get("name", "")
    if isinstance(args[0], dict):  # update_*(shard_obj, ...)
        return meta(args[0]).get("namespace", ""), meta(args[0]).get("name", "")
    return args[1], args[0]  # create_template/create_workgroup(name, ns, ...)


class RogueResourceError(Exception):
    """A shard dependent exists without any owner reference (controller.go:494-499)."""


class ShardNotReadyError(Exception):
    """A shard's caches have not synced yet (native mode defers instead of blocking startup)."""


class ShardSyncError(Exception):
    """Aggregate of per-shard failures under failure isolation."""

    def __init__(self, failures: dict):
        self.failures = failures
        super().__init__("; ".join(f"{k}: {v}" for k, v in failures.items()))


# ---------------------------------------------------------------- equality helpers
def spec_matches(desired_spec, shard_obj: dict, desired_fp: int | None = None) -> bool:
    """reflect.DeepEqual(shard.Spec, template.Spec) — O(1) against a slim-cache digest.  `desired_fp`
    lets a multi-shard pass fingerprint the desired spec once."""
    fp = shard_obj.get(SLIM_FP)
    if fp is not None:
        want = desired_fp if desired_fp is not None else fingerprint(desired_spec)
        if want == fp[0]:
            return True
        wrote = shard_obj.get(SLIM_WROTE)  # the server rewrote our last write of exactly this spec
        return wrote is not None and wrote[0] == want
    return desired_spec == shard_obj.get("spec")


def data_matches(src: dict, shard_obj: dict, with_binary: bool) -> bool:
    """reflect.DeepEqual(src.Data, shard.Data) (+ binaryData in native mode)."""
    fp = shard_obj.get(SLIM_FP)
    if fp is not None:
        want = (fingerprint(src.get("data") or None),
                fingerprint(src.get("binaryData") or None) if with_binary else None)
        for got in (fp, shard_obj.get(SLIM_WROTE)):  # as stored, or as our last write of it meant it
            if got is not None and got[0] == want[0] and (not with_binary or got[1] == want[1]):
                return True
        return False
    if normalize_data(src.get("data")) != normalize_data(shard_obj.get("data")):
        return False
    return (not with_binary) or normalize_data(src.get("binaryData")) == normalize_data(shard_obj.get("binaryData"))


def slim_spec(obj: dict) -> dict:
    """Informer transform for shard templates/workgroups: keep metadata, replace spec by its digest."""
    out = {k: v for k, v in obj.items() if k not in ("spec", "status")}
    out[SLIM_FP] = (fingerprint(obj.get("spec")),)
    return out


def slim_data(obj: dict) -> dict:
    """Informer transform for shard secrets/configmaps: keep metadata/type, replace payloads by digests."""
    out = {k: v for k, v in obj.items() if k not in ("data", "binaryData", "stringData")}
    out[SLIM_FP] = (fingerprint(obj.get("data") or None), fingerprint(obj.get("binaryData") or None))
    return out


async def gather_all(coros) -> list:
    """asyncio.gather(..., return_exceptions=True) without Task overhead for the common single case."""
    coros = list(coros)
    if len(coros) == 1:
        try:
            return [await coros[0]]
        except asyncio.CancelledError:
            raise
        except Exception as e:  # noqa: BLE001
            return [e]
    return await asyncio.gather(*coros, return_exceptions=True)


def _shard_failure(e: BaseException, kind: str, name: str) -> dict:
    """Typed failure of one shard's step: a dependent's tag wins; a shard that has not synced names no object."""
    if isinstance(e, ShardNotReadyError):
        return F.from_exception(e)
    return F.from_exception(e, kind, name)


class ReconcileMixin:
    """Reconcile logic; mixed into `Controller` (which provides clients, listers, options)."""

    # ============================================================ status (controller.go:428-480)
    async def _write_status(self, rt, namespace: str, obj: dict, field_manager: str | None = None) -> dict:
        """UpdateStatus (compat: PUT with the cached resourceVersion, 409 on a concurrent edit) or, in
        native mode, a JSON merge PATCH of `.status` — the controller owns status, so a spec edit by a
        user racing with our status write no longer costs a conflict and a retry."""
        if self.options.patch_writes:
            return await self.client.patch(rt, namespace, meta(obj).get("name", ""), {"status": obj.get("status")},
                                           patch_type=PATCH_MERGE, field_manager=field_manager, subresource="status")
        return await self.client.update_status(rt, namespace, obj, field_manager=field_manager)

    def _carry_adoption(self, old: dict, new):
        """Keep a template's adoption mark (adoption_cache) across our own status write.

        A status write changes only `.status` — but native mode sends it as a merge PATCH without a
        resourceVersion precondition, so the response may already carry a user's spec edit made after our
        read (e.g. a new secretRef).  The mark moves to the response's version only when that version
        references the same Secrets/ConfigMaps; otherwise it is dropped and the next pass re-adopts."""
        if self.options.adoption_cache and isinstance(new, dict):
            om, nm = meta(old), meta(new)
            key = f"{C.KIND_TEMPLATE}/{om.get('namespace', '')}/{om.get('name', '')}"
            if self._adopted.get(key) == om.get("resourceVersion"):
                if om.get("uid") == nm.get("uid") and same_references(old, new):
                    self._adopted[key] = nm.get("resourceVersion")
                else:
                    self._adopted.pop(key, None)
        return new

    async def report_template_init_condition(self, template: dict) -> dict:
        status = template.get("status") or {}
        if not status.get("conditions"):
            name = meta(template).get("name", "")
            new = with_fields(template, status=dict(status, conditions=[
                ready_condition(now_rfc3339(), C.CONDITION_FALSE, f"Algorithm {q(name)} initializing")]))
            self._pass_wrote()
            res = await self._write_status(R.TEMPLATES, meta(template).get("namespace", ""), new,
                                           field_manager=C.FIELD_MANAGER)
            return self._carry_adoption(template, self._assume(self.template_informer, res))
        return template

    async def report_workgroup_init_condition(self, workgroup: dict) -> dict:
        status = workgroup.get("status") or {}
        if not status.get("conditions"):
            name = meta(workgroup).get("name", "")
            new = with_fields(workgroup, status=dict(status, conditions=[
                ready_condition(now_rfc3339(), C.CONDITION_FALSE, f"Workgroup {q(name)} initializing")]))
            self._pass_wrote()
            res = await self._write_status(R.WORKGROUPS, meta(workgroup).get("namespace", ""), new,
                                           field_manager=C.FIELD_MANAGER)
            return self._assume(self.workgroup_informer, res)
        return workgroup

    async def report_workgroup_synced_condition(self, workgroup: dict, ready: bool = True,
                                                message: str | None = None) -> dict:
        status = workgroup.get("status") or {}
        conds = list(status.get("conditions") or [])
        name = meta(workgroup).get("name", "")
        msg = message or f"Workgroup {q(name)} ready"
        conds[0] = ready_condition(conds[0].get("lastTransitionTime", ""),
                                   C.CONDITION_TRUE if ready else C.CONDITION_FALSE, msg)
        new_status = dict(status, conditions=conds)
        if new_status != status:
            conds[0] = dict(conds[0], lastTransitionTime=now_rfc3339())
            self._pass_wrote()
            res = await self._write_status(R.WORKGROUPS, meta(workgroup).get("namespace", ""),
                                           with_fields(workgroup, status=new_status), field_manager=C.FIELD_MANAGER)
            return self._assume(self.workgroup_informer, res)
        return workgroup

    @staticmethod
    def _template_synced_status(template: dict, secrets: list, configmaps: list, shards: list, ready: bool = True,
                                message: str | None = None) -> tuple:
        """(current status, status after a synced report, its conditions list) — equal statuses mean no write."""
        status = template.get("status") or {}
        conds = list(status.get("conditions") or [])
        name = meta(template).get("name", "")
        msg = message or f"Algorithm {q(name)} ready"
        conds[0] = ready_condition(conds[0].get("lastTransitionTime", ""),
                                   C.CONDITION_TRUE if ready else C.CONDITION_FALSE, msg)
        new_status = dict(status, conditions=conds, syncedSecrets=list(secrets),
                          syncedConfigurations=list(configmaps), syncedToClusters=list(shards))
        return status, new_status, conds

    async def report_template_synced_condition(self, template: dict, secrets: list, configmaps: list, shards: list,
                                               ready: bool = True, message: str | None = None) -> dict:
        status, new_status, conds = self._template_synced_status(template, secrets, configmaps, shards, ready,
                                                                 message)
        if new_status != status:
            conds[0] = dict(conds[0], lastTransitionTime=now_rfc3339())
            self._pass_wrote()
            res = await self._write_status(R.TEMPLATES, meta(template).get("namespace", ""),
                                           with_fields(template, status=new_status), field_manager=C.FIELD_MANAGER)
            return self._carry_adoption(template, self._assume(self.template_informer, res))
        return template

    # ============================================================ ownership (controller.go:482-502)
    def is_missing_ownership(self, obj: dict, owner: dict, kind: str, template: dict | None = None,
                             shard_name: str = "") -> bool:
        refs = meta(obj).get("ownerReferences") or []
        if refs:
            owner_uid = meta(owner).get("uid", "") or ""
            for r in refs:
                if r.get("kind") == C.TEMPLATE_KIND and (r.get("uid", "") or "") == owner_uid:
                    return False
            return True
        msg = C.MESSAGE_RESOURCE_EXISTS.format(q(meta(obj).get("name", "")))
        if self.options.rogue_event_on_template and template is not None:
            # native: report on the controller-side template the user owns, naming the shard and kind
            self.recorder.event(template, C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_EXISTS,
                                f"{kind} {msg} (shard {q(shard_name)})", kind=C.TEMPLATE_KIND)
        else:
            # The reference records this against the *shard* object into the controller cluster (controller.go:497).
            self.recorder.event(obj, C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_EXISTS, msg, kind=kind)
        raise RogueResourceError(msg)

    # ============================================================ adoption (controller.go:647-695)
    async def adopt_references(self, template: dict) -> None:
        ns = meta(template).get("namespace", "")
        tname = meta(template).get("name", "")
        tuid = meta(template).get("uid", "") or ""
        pending = []
        for rt, names, lister, informer in ((R.SECRETS, secret_names(template), self.secret_lister,
                                             self.secret_informer),
                                            (R.CONFIGMAPS, configmap_names(template), self.configmap_lister,
                                             self.configmap_informer)):
            for nm in names:
                ref = lister.try_get(ns, nm)
                if ref is None and informer.owner_filter is not None:
                    # a partitioned coordinator may have dropped it off the wire (owned only by other
                    # partitions' templates when it arrived): read it once
                    try:
                        await self._fetch_filtered(informer, rt, ns, nm)
                    except E.NotFound:
                        pass
                    ref = lister.try_get(ns, nm)
                if ref is None:
                    self.recorder.event(template, C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_MISSING,
                                        C.MESSAGE_RESOURCE_MISSING.format(q(nm), q(tname)), kind=C.TEMPLATE_KIND)
                    lister.get(ns, nm)  # raises the typed NotFound
                if self.options.controller_adoption and not is_owned_by_uid(ref, tuid):
                    m = dict(meta(ref))
                    m["ownerReferences"] = list(m.get("ownerReferences") or []) + [template_owner_ref(template)]
                    args = (rt, ns, with_fields(ref, metadata=m), template, nm, informer)
                    if self.options.concurrent_dependents:
                        pending.append(args)  # validate every reference first, then write concurrently
                    else:
                        await self._adopt_one(*args)
        if pending:
            await self._gather_raise([self._adopt_one(*a) for a in pending])

    async def _adopt_one(self, rt, ns, obj, template, nm, informer):
        self._pass_wrote()
        try:
            if self.options.patch_writes:
                # strategic merge on ownerReferences (patchMergeKey=uid) appends without a resourceVersion race
                res = await self.client.patch(rt, ns, nm, {"metadata": {"ownerReferences": [template_owner_ref(template)]}},
                                              patch_type=PATCH_STRATEGIC, field_manager=C.FIELD_MANAGER)
            else:
                res = await self.client.update(rt, ns, obj)
            self._assume(informer, res)
        except Exception as e:  # noqa: BLE001
            self.recorder.event(template, C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_SYNC_ERROR,
                                C.MESSAGE_RESOURCE_OPERATION_FAILED.format(q(nm), q(meta(template).get("name", "")),
                                                                          e), kind=C.TEMPLATE_KIND)
            raise

    @staticmethod
    async def _gather_raise(jobs: list) -> None:
        res = await asyncio.gather(*jobs, return_exceptions=True)
        jobs.clear()
        for r in res:
            if isinstance(r, BaseException):
                raise r

    # ============================================================ templates (controller.go:761-845)
    async def sync_template(self, namespace: str, name: str) -> None:
        self._begin_pass()
        template = self.template_lister.try_get(namespace, name)
        if template is None:
            log.debug("NexusAlgorithmTemplate %s/%s referenced by item in work queue no longer exists",
                      namespace, name)
            self._adopted.pop(f"{C.KIND_TEMPLATE}/{namespace}/{name}", None)
            if self.role == "coordinator":
                self.reports.pop(f"{C.KIND_TEMPLATE}/{namespace}/{name}")
                self._failure_events.pop(f"{C.KIND_TEMPLATE}/{namespace}/{name}", None)
                self._inline_status_ok.pop(f"{C.KIND_TEMPLATE}/{namespace}/{name}", None)
                self._pending_event.discard(f"{C.KIND_TEMPLATE}/{namespace}/{name}")
            elif self.options.queued_deletes:
                await self.propagate_template_delete(namespace, name)
            return
        if self.role == "executor":
            await self._executor_sync_template(template)
            return
        template = await self.report_template_init_condition(template)
        if self.options.adoption_cache:
            key = f"{C.KIND_TEMPLATE}/{namespace}/{name}"
            rv = meta(template).get("resourceVersion")
            if self._adopted.get(key) != rv:
                # A dependent event during the awaits below (our ownerRef removed, the Secret re-created)
                # pops this token in `_on_dependent`; the mark is stored only if nothing invalidated it.
                token = object()
                self._adopted[key] = token
                await self.adopt_references(template)
                if self._adopted.get(key) is token:
                    self._adopted[key] = rv
        else:
            await self.adopt_references(template)
        if self.role == "coordinator":
            await self._coordinator_finish(C.KIND_TEMPLATE, template)
            return

        shard_names = self.shard_names()
        spec = template.get("spec")
        spec_fp = fingerprint(spec) if self.options.slim_shard_cache else None
        if self.options.concurrent_fanout:
            results = await gather_all(self._sync_template_to_shard(template, s, spec_fp) for s in self.shards)
            failures = {s.name: r for s, r in zip(self.shards, results) if isinstance(r, BaseException)}
            for r in failures.values():
                if isinstance(r, asyncio.CancelledError):
                    raise r
            if failures:
                if not self.options.shard_failure_isolation:
                    raise next(iter(failures.values()))
                ok = [n for n in shard_names if n not in failures]
                await self.report_template_synced_condition(
                    template, *dependent_names(template), ok, ready=False,
                    message=F.status_message(f"Algorithm {q(name)}", {
                        s: _shard_failure(e, C.TEMPLATE_KIND, name) for s, e in failures.items()}))
                raise ShardSyncError(failures)
        else:
            for shard in self.shards:
                await self._sync_template_to_shard(template, shard, spec_fp)

        template = await self.report_template_synced_condition(template, *dependent_names(template),
                                                               shard_names)
        if self.options.event_on_noop or self._last_pass_wrote():
            self.recorder.event(template, C.EVENT_TYPE_NORMAL, C.SUCCESS_SYNCED,
                                C.MESSAGE_RESOURCE_SYNCED.format("NexusAlgorithmTemplate"), kind=C.TEMPLATE_KIND)

    async def _executor_sync_template(self, template: dict) -> None:
        """Executor role: fan out to this process's shards only and report to the coordinator."""
        ns, name = meta(template).get("namespace", ""), meta(template).get("name", "")
        # the coordinator adopts; an executor only refuses to write when a reference is missing (as adoption would)
        secrets, configmaps = dependent_names(template)
        for rt, names, lister, informer in ((R.SECRETS, secrets, self.secret_lister, self.secret_informer),
                                            (R.CONFIGMAPS, configmaps, self.configmap_lister,
                                             self.configmap_informer)):
            for nm in names:
                if lister.try_get(ns, nm) is None:
                    await self._executor_fetch_reference(informer, rt, ns, nm, template)
        spec_fp = fingerprint(template.get("spec")) if len(self.shards) > 1 and self.options.slim_shard_cache else None
        results = await gather_all(self._sync_template_to_shard(template, s, spec_fp) for s in self.shards)
        failures = {}
        for s, r in zip(self.shards, results):
            if isinstance(r, asyncio.CancelledError):
                raise r
            if isinstance(r, BaseException):
                failures[s.name] = r
        self._report(C.KIND_TEMPLATE, ns, name, template,
                     {s.name: (_shard_failure(failures[s.name], C.TEMPLATE_KIND, name) if s.name in failures else None)
                      for s in self.shards})
        if failures:
            raise ShardSyncError(failures)

    async def _executor_fetch_reference(self, informer, rt, ns: str, nm: str, template: dict) -> None:
        """A referenced Secret/ConfigMap this executor has not received: with the watch relay, ask the
        coordinator for it (it may have been routed to another partition while only other partitions'
        templates owned it) as the C++ executor does; otherwise read it once.  The pass then fails without a
        report and retries with backoff: the coordinator's adoption pass, which reads its own cache, is the
        authority on a missing reference (ErrResourceMissing), and a relay that is a line behind must not flap
        the status to Ready=False."""
        if self.need is not None:
            self.need(2 if rt is R.SECRETS else 3, f"{ns}/{nm}")
        try:
            await self._fetch_filtered(informer, rt, ns, nm)
        except E.NotFound as e:
            raise F.mark(e, rt.kind, nm, F.REFERENCE_MISSING)

    async def _fetch_filtered(self, informer, rt, ns: str, name: str) -> None:
        """A referenced dependent missing from a partition-filtered cache may have been dropped off the wire
        while it was owned only by other partitions' templates (a template of ours started referencing it
        since): read it once; from now on the reference keeps its watch events flowing to this cache.
        NotFound propagates as the missing-reference error it is."""
        if informer.owner_filter is None:
            informer.lister.get(ns, name)  # raises the typed NotFound
            return
        obj = await self.client.get(rt, ns, name)
        if informer.lister.try_get(ns, name) is None:  # the watch may have delivered it meanwhile
            informer.store.upsert(obj)

    async def _coordinator_finish(self, kind: str, obj: dict) -> None:
        """Coordinator role: turn the executors' per-shard reports into the status condition."""
        ns, name = meta(obj).get("namespace", ""), meta(obj).get("name", "")
        key = f"{kind}/{ns}/{name}"
        results = self.shard_readiness(key, obj)
        if results is None:
            return  # some shard has not reported on this version yet; its report re-enqueues the key
        failures = {s: F.normalize(e) for s, e in results.items() if e}
        ok = [s for s in self.all_shard_names if not results[s]]
        is_template = kind == C.KIND_TEMPLATE
        if failures:
            what = f"Algorithm {q(name)}" if is_template else f"Workgroup {q(name)}"
            msg = F.status_message(what, failures)
            if is_template:
                self._record_failure_events(key, obj, failures)
                await self.report_template_synced_condition(obj, *dependent_names(obj), ok,
                                                            ready=False, message=msg)
            else:
                await self.report_workgroup_synced_condition(obj, ready=False, message=msg)
            return
        self._failure_events.pop(key, None)
        if is_template:
            obj = await self.report_template_synced_condition(obj, *dependent_names(obj), ok)
        else:
            obj = await self.report_workgroup_synced_condition(obj)
        if key in self._pending_event or self._last_pass_wrote() or self.options.event_on_noop:
            self._pending_event.discard(key)
            kind_name = C.TEMPLATE_KIND if is_template else C.WORKGROUP_KIND
            self.recorder.event(obj, C.EVENT_TYPE_NORMAL, C.SUCCESS_SYNCED,
                                C.MESSAGE_RESOURCE_SYNCED.format(kind_name), kind=kind_name)

    def _record_failure_events(self, key: str, template: dict, failures: dict) -> None:
        """Coordinator: the Warning Events the in-process reconcile records where a shard write fails
        (controller.go:497,525-557,587-619), from the executors' typed failures.  Recorded once per distinct
        failure and shard: a backoff retry that fails the same way again changes nothing to announce (the
        report table does not even complete a repeat of an identical report set), and the memo also covers
        a set that completes again because *another* shard's result changed."""
        seen = self._failure_events.setdefault(key, {})  # shard -> (signature, failure): also /debug/state
        for shard in sorted(failures):
            f = failures[shard]
            sig = F.signature(f)
            if seen.get(shard, (None,))[0] == sig:
                continue
            seen[shard] = (sig, f)
            for etype, reason, message in F.events(f, meta(template).get("name", ""), shard):
                self.recorder.event(template, etype, reason, message, kind=C.TEMPLATE_KIND)
        for shard in [s for s in seen if s not in failures]:
            del seen[shard]

    def finish_inline(self, key: str) -> bool:
        """Coordinator: the pass a complete set of executor reports would run, done synchronously when it can
        only end in the `Synced` Event — the template exists, is initialised and adopted at this version, every
        shard succeeded and the status already says so.  Saves the queue round trip, the worker hand-off and
        the pass preamble for the common case.  False (nothing done) when a real pass is needed: a status or
        adoption write, a failure to report, a deletion, or a pass already queued or running for the key."""
        return not self.finish_inline_many((key,))

    def finish_inline_many(self, keys) -> list:
        """`finish_inline` over a batch of keys; returns the keys that need a real pass.  The native report
        table decides the common case (a slim template whose status was verified before) without running
        Python per key; what it cannot decide goes through `_finish_inline_py`, the specification."""
        if not self.ready.is_set() or self.queue.shutting_down() or not self.options.adoption_cache:
            return list(keys)  # workers not running (standby, shutdown, lost Lease): nothing may be written
        fb = getattr(self.reports, "finish_batch", None)
        core = getattr(self.queue, "core", None)
        if fb is None or core is None:
            return self._finish_inline_py(keys)
        store = self.template_informer.store
        rest, verify, events, done, superseded = fb(
            keys, store._items, store._assumed, self._adopted, self._inline_status_ok, self.all_shard_names, core,
            self._pending_event, self.options.event_on_noop)
        st = self.stats
        st["inline_superseded"] += superseded
        done += len(events)
        if events:
            record, msg = self.recorder.event, _SYNCED_MESSAGE
            for template in events:
                record(template, C.EVENT_TYPE_NORMAL, C.SUCCESS_SYNCED, msg, kind=C.TEMPLATE_KIND)
        if done:
            st["reconciles"] += done
            st["inline_finishes"] += done
            self.metrics.gauge_duration(C.RECONCILE_LATENCY_METRIC, time.monotonic())
        if verify:
            rest.extend(self._finish_inline_py(verify))
        return rest

    def _finish_inline_py(self, keys) -> list:
        """finish_inline_many, one key at a time in Python (the loop invariants read once)."""
        busy = self.queue.busy
        get = self.template_informer.store.get
        adopted = self._adopted
        ready_ok = self.reports.ready_ok
        memos = self._inline_status_ok
        pending_event = self._pending_event
        event_on_noop = self.options.event_on_noop
        shards = self.all_shard_names
        kind_template = C.KIND_TEMPLATE
        st = self.stats
        rest = []
        done = 0
        for key in keys:
            try:
                kind, ns, name = key.split("/", 2)
                if kind != kind_template or busy(key):
                    rest.append(key)
                    continue
                template = get(ns, name)
                if template is None:
                    rest.append(key)
                    continue
                status = template.get("status") or {}
                conds = status.get("conditions")
                m = template.get("metadata") or {}
                if not conds or adopted.get(key) != m.get("resourceVersion"):
                    rest.append(key)
                    continue
                ok = ready_ok(key, m.get("uid") or "", m.get("generation") or 0)
                if ok is None:
                    # A newer version (the next wave) reached the cache between the last report and this
                    # flush.  It is initialised and adopted, so the pass would stop at the readiness check,
                    # exactly as the early pass `_on_crd_update` skips: the new version's last report brings
                    # the key back.
                    st["inline_superseded"] += 1
                    continue
                if not ok:
                    rest.append(key)
                    continue
                # report_template_synced_condition would leave the status as it is (no write) exactly when the
                # Ready condition and the three synced lists already hold what it would set.  That depends only
                # on the status, the references and the shard list: a new template version (the next wave)
                # with an equal status and equal references reuses the last verdict — of a slim template, two
                # int compares of the digests of their texts.
                spec = template.get("spec") or {}
                sfp, rfp = template.get(SLIM_STATUS_FP), spec.get("_rfp")
                if sfp is not None and rfp is not None:
                    status_id, refs = sfp, rfp
                else:
                    status_id, refs = status, (spec.get("runtimeEnvironment") or {}).get("mappedEnvironmentVariables")
                memo = memos.get(key)
                if memo is None or memo[2] is not shards or memo[0] != status_id or memo[1] != refs:
                    secrets, configmaps = dependent_names(template)
                    c0 = conds[0]
                    if c0 != ready_condition(c0.get("lastTransitionTime", ""), C.CONDITION_TRUE,
                                             f"Algorithm {q(name)} ready") \
                            or status.get("syncedSecrets") != secrets \
                            or status.get("syncedConfigurations") != configmaps \
                            or status.get("syncedToClusters") != shards:
                        rest.append(key)
                        continue
                    memos[key] = (status_id, refs, shards)
                done += 1
                if key in pending_event or event_on_noop:
                    pending_event.discard(key)
                    self.recorder.event(template, C.EVENT_TYPE_NORMAL, C.SUCCESS_SYNCED,
                                        C.MESSAGE_RESOURCE_SYNCED.format(C.TEMPLATE_KIND), kind=C.TEMPLATE_KIND)
            except Exception:  # noqa: BLE001 — the queued pass will hit (and report) the same problem
                log.exception("inline finish of %s failed; queueing a pass", key)
                rest.append(key)
        if done:
            st["reconciles"] += done
            st["inline_finishes"] += done
            # a reconcile done in place takes no time: one gauge per batch (an aggregated gauge keeps the last)
            self.metrics.gauge_duration(C.RECONCILE_LATENCY_METRIC, time.monotonic())
        return rest

    async def _sync_template_to_shard(self, template: dict, shard, spec_fp) -> None:
        if self.options.wait_for_shards_timeout is not None and not shard.has_synced():
            raise ShardNotReadyError(f"shard {shard.name} caches not synced")
        ns = meta(template).get("namespace", "")
        name = meta(template).get("name", "")
        spec = template.get("spec")
        shard_template = shard.template_lister.try_get(ns, name)
        update = update_error = None
        if self.options.server_side_apply:
            if shard_template is None or not spec_matches(spec, shard_template, spec_fp):
                self._pass_wrote()
                try:
                    shard_template = await shard.apply_template(name, ns, spec, C.FIELD_MANAGER)
                except Exception as e:  # noqa: BLE001 — as for the update below: the UID is known
                    if shard_template is None or not self.options.dependents_despite_template_failure:
                        raise
                    update_error = e
        elif shard_template is not None and not spec_matches(spec, shard_template, spec_fp):
            log.debug("Content changed for NexusAlgorithmTemplate %s, updating", name)
            update = self._write(shard, "update_template", shard.template_informer, R.TEMPLATES,
                                 shard_template, spec, C.FIELD_MANAGER)
            if not self.options.concurrent_dependents:
                try:
                    shard_template = await update
                except Exception as e:  # noqa: BLE001
                    if not self.options.dependents_despite_template_failure:
                        raise
                    # native: the shard template keeps its UID, which is all its dependents' ownerRefs need,
                    # so a refused update (a 422, say) does not hold back the new Secret/ConfigMap data; the
                    # pass still fails with the template's error (README "Modes")
                    update_error = e
                update = None
            # native: an update keeps the shard template's UID, so its dependents go out alongside it
            # instead of one round trip later (controller.go:790-831 is strictly sequential)
        elif shard_template is None:
            log.debug("Algorithm %s not found in shard %s, creating", name, shard.name)
            shard_template = await self._write(shard, "create_template", shard.template_informer, R.TEMPLATES,
                                               name, ns, spec, C.FIELD_MANAGER)
        if self.options.concurrent_dependents:
            # dependents need the shard template's UID for their ownerRefs, so they go after it — all at once
            # a shard template still being updated, or whose apply was refused, carries the old references
            holder = template if (update is not None or update_error is not None or SLIM_FP in shard_template
                                  or shard_template.get("spec") is None) else shard_template
            secrets, configmaps = dependent_names(holder)
            jobs = [self._sync_dependent(R.SECRETS, template, shard_template, shard, n) for n in secrets]
            jobs += [self._sync_dependent(R.CONFIGMAPS, template, shard_template, shard, n) for n in configmaps]
            if update is not None:
                jobs.insert(0, update)
            for r in await gather_all(jobs):
                if isinstance(r, BaseException):
                    raise r
            if update_error is not None:  # the dependents went out; the pass still fails with the apply's error
                raise update_error
        else:
            # after a refused update the shard template still has the old spec: the references are the source's
            holder = template if update_error is not None else None
            await self._sync_dependents_to_shard(R.SECRETS, template, shard_template, shard, holder)
            await self._sync_dependents_to_shard(R.CONFIGMAPS, template, shard_template, shard, holder)
            if update_error is not None:
                raise update_error

    async def _write(self, shard, op: str, informer, rt, *args):
        """Issue a shard write; in native mode resolve create/update races by refetching."""
        self._pass_wrote()
        try:
            return await getattr(shard, op)(*args)
        except (E.AlreadyExists, E.Conflict) as e:
            if not self.options.tolerate_write_races:
                raise
            # Our cache was stale: fetch the live object, publish it, let the caller continue from it.
            ns, nm = _write_target(op, args)
            live = await shard.client.get(rt, ns, nm)
            informer.store.assume(live)
            if isinstance(e, E.Conflict) and op.startswith("update"):
                retry_args = (informer.store.get(ns, nm) or live,) + tuple(args[1:])
                return await getattr(shard, op)(*retry_args)
            return informer.store.get(ns, nm) or live

    async def _sync_dependents_to_shard(self, rt, template: dict, shard_template: dict, shard,
                                        holder: dict | None = None) -> None:
        """syncSecretsToShard / syncConfigMapsToShard (controller.go:504-626)."""
        is_secret = rt is R.SECRETS
        # GetSecretNames() is read from the shard template (controller.go:505); its spec equals the
        # controller's after create/update.  A slim-cache shard template carries no spec: use the source.
        if holder is None:
            holder = template if (SLIM_FP in shard_template or shard_template.get("spec") is None) \
                else shard_template
        names = secret_names(holder) if is_secret else configmap_names(holder)
        if self.options.concurrent_dependents and len(names) > 1:
            res = await asyncio.gather(*(self._sync_dependent(rt, template, shard_template, shard, n) for n in names),
                                       return_exceptions=True)
            for r in res:
                if isinstance(r, BaseException):
                    raise r
        else:
            for n in names:
                await self._sync_dependent(rt, template, shard_template, shard, n)

    def _dependent_failed(self, template: dict, kind: str, dep_name: str, e: BaseException) -> BaseException:
        """Warning ErrResourceSyncError on the template (controller.go:525,546,557); returns `e` to raise,
        tagged with the dependent it concerns (the typed failure an executor reports, `failures.py`)."""
        F.mark(e, kind, dep_name)
        self.recorder.event(template, C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_SYNC_ERROR,
                            C.MESSAGE_RESOURCE_OPERATION_FAILED.format(q(dep_name), q(meta(template).get("name", "")),
                                                                      e), kind=C.TEMPLATE_KIND)
        return e

    async def _put_dependent(self, shard, rt, src: dict, obj: dict, data, owner, with_binary: bool):
        """UpdateSecret / UpdateConfigMap (X8f) of a shard dependent, race-tolerant in native mode."""
        is_secret = rt is R.SECRETS
        args = (obj, data, owner, C.FIELD_MANAGER)
        if with_binary:
            args = args + (normalize_data(src.get("binaryData")),)
        if self.options.sync_dependent_metadata and data is not None:
            args = args + ((None,) if not is_secret and not with_binary else ()) + (shard.dependent_metadata(src),)
        if self.options.tolerate_write_races:
            informer = shard.secret_informer if is_secret else shard.configmap_informer
            return await self._write(shard, "update_secret" if is_secret else "update_configmap", informer, rt,
                                     *args)
        self._pass_wrote()
        return await (shard.update_secret if is_secret else shard.update_configmap)(*args)

    async def _sync_dependent(self, rt, template: dict, shard_template: dict, shard, dep_name: str) -> None:
        is_secret = rt is R.SECRETS
        kind = rt.kind
        tm = meta(template)
        ns = tm.get("namespace", "")
        lister = self.secret_lister if is_secret else self.configmap_lister
        src = lister.try_get(ns, dep_name)
        if src is None:
            self.recorder.event(template, C.EVENT_TYPE_WARNING, C.ERR_RESOURCE_MISSING,
                                C.MESSAGE_RESOURCE_MISSING.format(q(dep_name), q(tm.get("name", ""))),
                                kind=C.TEMPLATE_KIND)
            try:
                lister.get(ns, dep_name)  # raises NotFound
            except E.NotFound as e:
                raise F.mark(e, kind, dep_name, F.REFERENCE_MISSING)
        shard_ns = meta(shard_template).get("namespace", "")
        shard_lister = shard.secret_lister if is_secret else shard.configmap_lister
        shard_obj = shard_lister.try_get(shard_ns, meta(src).get("name", ""))
        opts = self.options
        with_binary = opts.sync_binary_data and not is_secret
        shard_informer = shard.secret_informer if is_secret else shard.configmap_informer
        create = "create_secret" if is_secret else "create_configmap"
        if opts.server_side_apply:
            # Every template's pass applies with the same field manager, and an apply drops the ownerRef entries
            # its manager applied before and omits now.  So an apply over a known copy carries that copy's
            # template ownerRefs and its resourceVersion (a concurrent change → 409 → once more from the live
            # copy).  A ref lost anyway — two passes creating the same copy at once from empty caches — is
            # repaired from the shard watch (Controller._register_shard_handlers).
            try:
                for attempt in range(2):
                    if shard_obj is not None:
                        missing_owner = self.is_missing_ownership(shard_obj, shard_template, kind, template,
                                                                  shard.name)  # rogue → error
                        if is_secret and opts.sync_secret_type and \
                                (src.get("type") or "Opaque") != (shard_obj.get("type") or "Opaque"):
                            # Secret.type is immutable, so an apply cannot change it: replace the copy
                            self._pass_wrote()
                            await self._delete_one(shard, lambda o: shard.delete_dependent(R.SECRETS, o), shard_obj)
                            shard_obj = None
                        elif not missing_owner and data_matches(src, shard_obj, with_binary) and \
                                (not opts.sync_dependent_metadata or shard.dependent_metadata_matches(src, shard_obj)):
                            return
                    self._pass_wrote()
                    try:
                        res = await shard.apply_dependent(rt, shard_template, src, C.FIELD_MANAGER, live=shard_obj)
                        if shard_obj is None and isinstance(res, dict):
                            # applied without a view of the copy: if it existed, refs may have been dropped
                            self.repair_lost_owners(shard, "secret" if is_secret else "configmap", res)
                        return
                    except E.Conflict:
                        if attempt:
                            raise
                    live = await shard.client.get(rt, shard_ns, dep_name)
                    shard_informer.store.assume(live)
                    shard_obj = shard_informer.store.get(shard_ns, dep_name) or live
            except Exception as e:  # noqa: BLE001
                raise self._dependent_failed(template, kind, dep_name, e)
            return
        if shard_obj is None:
            try:
                shard_obj = await self._write(shard, create, shard_informer, rt, shard_template, src,
                                              C.FIELD_MANAGER)
            except Exception as e:  # noqa: BLE001
                raise self._dependent_failed(template, kind, dep_name, e)
        try:
            missing_owner = self.is_missing_ownership(shard_obj, shard_template, kind, template, shard.name)
        except RogueResourceError as e:
            raise self._dependent_failed(template, kind, dep_name, e)
        if is_secret and opts.sync_secret_type and \
                (src.get("type") or "Opaque") != (shard_obj.get("type") or "Opaque"):
            # Secret.type is immutable: replace the shard copy (other owners re-add their refs on their passes)
            try:
                self._pass_wrote()
                await self._delete_one(shard, lambda o: shard.delete_dependent(R.SECRETS, o), shard_obj)
                shard_obj = await self._write(shard, "create_secret", shard_informer, rt, shard_template, src,
                                              C.FIELD_MANAGER)
            except Exception as e:  # noqa: BLE001
                raise self._dependent_failed(template, kind, dep_name, e)
            return
        differs = not data_matches(src, shard_obj, with_binary)
        if opts.sync_dependent_metadata and not differs and not shard.dependent_metadata_matches(src, shard_obj):
            differs = True  # labels/annotations only: one PUT carries them (with the unchanged data)
        try:
            slim = SLIM_FP in shard_obj
            if opts.single_put_dependents or slim:
                if differs or missing_owner:
                    await self._put_dependent(shard, rt, src, shard_obj,
                                              normalize_data(src.get("data")) if (differs or slim) else None,
                                              shard_template if missing_owner else None, with_binary)
            else:
                if differs:
                    log.debug("Content changed for %s %s, updating", kind, dep_name)
                    await self._put_dependent(shard, rt, src, shard_obj, src.get("data"), None, with_binary)
                if missing_owner:
                    log.debug("Ownership missing for %s %s, updating", kind, dep_name)
                    # The reference re-uses the pre-update object here (controller.go:552,614).
                    await self._put_dependent(shard, rt, src, shard_obj, None, shard_template, with_binary)
        except Exception as e:  # noqa: BLE001
            raise self._dependent_failed(template, kind, dep_name, e)

    async def propagate_template_delete(self, namespace: str, name: str) -> None:
        """Level-triggered shard delete (native `queued_deletes`): retried through the queue."""
        key = (namespace, name)
        explicit = key in self._pending_deletes
        jobs = []
        for shard in self.shards:
            st = shard.template_lister.try_get(namespace, name)
            if st is None:
                continue
            if not explicit and not self._is_ours(st):
                continue
            jobs.append(self._delete_one(shard, shard.delete_template, st))
        if jobs:
            res = await asyncio.gather(*jobs, return_exceptions=True)
            errs = [r for r in res if isinstance(r, BaseException)]
            if errs:
                raise errs[0]
        self._pending_deletes.discard(key)

    async def propagate_workgroup_delete(self, namespace: str, name: str) -> None:
        key = (namespace, name)
        explicit = key in self._pending_workgroup_deletes
        jobs = []
        for shard in self.shards:
            sw = shard.workgroup_lister.try_get(namespace, name)
            if sw is None or (not explicit and not self._is_ours(sw)):
                continue
            jobs.append(self._delete_one(shard, shard.delete_workgroup, sw))
        if jobs:
            res = await asyncio.gather(*jobs, return_exceptions=True)
            errs = [r for r in res if isinstance(r, BaseException)]
            if errs:
                raise errs[0]
        self._pending_workgroup_deletes.discard(key)

    async def _delete_one(self, shard, fn, obj) -> None:
        if self.options.wait_for_shards_timeout is not None and not shard.has_synced():
            raise ShardNotReadyError(f"shard {shard.name} caches not synced")
        try:
            await fn(obj)
        except E.NotFound:
            pass

    def _is_ours(self, obj: dict) -> bool:
        lbl = meta(obj).get("labels") or {}
        return lbl.get(C.LABEL_CONFIGURATION_OWNER) == self.alias and \
            lbl.get(C.LABEL_CONTROLLER_APP) == C.CONTROLLER_AGENT_NAME

    # ============================================================ workgroups (controller.go:697-756)
    async def sync_workgroup(self, namespace: str, name: str) -> None:
        self._begin_pass()
        workgroup = self.workgroup_lister.try_get(namespace, name)
        if workgroup is None:
            log.debug("NexusAlgorithmWorkgroup %s/%s referenced by item in work queue no longer exists",
                      namespace, name)
            if self.role == "coordinator":
                self.reports.pop(f"{C.KIND_WORKGROUP}/{namespace}/{name}")
                self._pending_event.discard(f"{C.KIND_WORKGROUP}/{namespace}/{name}")
            elif self.options.propagate_workgroup_deletes:
                await self.propagate_workgroup_delete(namespace, name)
            return
        if self.role == "executor":
            results = await gather_all(self._sync_workgroup_to_shard(workgroup, s) for s in self.shards)
            failures = {s.name: r for s, r in zip(self.shards, results) if isinstance(r, BaseException)}
            self._report(C.KIND_WORKGROUP, namespace, name, workgroup,
                         {s.name: (_shard_failure(failures[s.name], C.WORKGROUP_KIND, name)
                                   if s.name in failures else None) for s in self.shards})
            if failures:
                raise ShardSyncError(failures)
            return
        workgroup = await self.report_workgroup_init_condition(workgroup)
        if self.role == "coordinator":
            await self._coordinator_finish(C.KIND_WORKGROUP, workgroup)
            return
        if self.options.concurrent_fanout:
            results = await gather_all(self._sync_workgroup_to_shard(workgroup, s) for s in self.shards)
            failures = {s.name: r for s, r in zip(self.shards, results) if isinstance(r, BaseException)}
            if failures:
                if self.options.shard_failure_isolation:
                    await self.report_workgroup_synced_condition(
                        workgroup, ready=False,
                        message=F.status_message(f"Workgroup {q(name)}", {
                            s: _shard_failure(e, C.WORKGROUP_KIND, name) for s, e in failures.items()}))
                    raise ShardSyncError(failures)
                raise next(iter(failures.values()))
        else:
            for shard in self.shards:
                await self._sync_workgroup_to_shard(workgroup, shard)
        workgroup = await self.report_workgroup_synced_condition(workgroup)
        if self.options.event_on_noop or self._last_pass_wrote():
            self.recorder.event(workgroup, C.EVENT_TYPE_NORMAL, C.SUCCESS_SYNCED,
                                C.MESSAGE_RESOURCE_SYNCED.format("NexusAlgorithmWorkgroup"), kind=C.WORKGROUP_KIND)

    async def _sync_workgroup_to_shard(self, workgroup: dict, shard) -> None:
        if self.options.wait_for_shards_timeout is not None and not shard.has_synced():
            raise ShardNotReadyError(f"shard {shard.name} caches not synced")
        ns = meta(workgroup).get("namespace", "")
        name = meta(workgroup).get("name", "")
        spec = workgroup.get("spec")
        sw = shard.workgroup_lister.try_get(ns, name)
        if self.options.server_side_apply:
            if sw is None or not spec_matches(spec, sw):
                self._pass_wrote()
                await shard.apply_workgroup(name, ns, spec, C.FIELD_MANAGER)
        elif sw is not None and not spec_matches(spec, sw):
            await self._write(shard, "update_workgroup", shard.workgroup_informer, R.WORKGROUPS, sw, spec,
                              C.FIELD_MANAGER)
        elif sw is None:
            await self._write(shard, "create_workgroup", shard.workgroup_informer, R.WORKGROUPS, name, ns, spec,
                              C.FIELD_MANAGER)

    def shard_names(self) -> list[str]:
        return [s.name for s in self.shards]
