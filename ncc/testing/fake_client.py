"""In-process fake cluster client with a recorded action log.

The analogue of client-go's `fake.NewSimpleClientset` + `testing.Fake.Actions()` that the
reference's unit tests are built on (controller_test.go:492-498, 383-466).  Every call is
appended to `actions` *before* it is applied, with a deep copy of the request object, so a
test can assert the exact ordered sequence of writes a reconcile issued per client — and,
filtering by API group, per typed clientset as the reference does (four clients:
controller-nexus, controller-kube, shard-nexus, shard-kube; controller_test.go:632-635).

Reactors (`prepend_reactor`) allow error injection, like client-go's `PrependReactor`.
"""
from __future__ import annotations

import asyncio
from dataclasses import dataclass, field
from typing import Any, Callable

from ..aio import wait_timeout
from ..api.objects import deep_copy
from ..api.resources import ResourceType
from ..fakeapi.storage import ClusterState
from ..kube.client import PATCH_MERGE, KubeClient, WatchEvent


@dataclass
class Action:
    verb: str
    resource: ResourceType
    namespace: str
    name: str = ""
    subresource: str = ""
    obj: Any = None
    patch: Any = None
    patch_type: str = ""
    extra: dict = field(default_factory=dict)

    @property
    def group(self) -> str:
        return self.resource.group_key

    def __repr__(self) -> str:
        sub = f"/{self.subresource}" if self.subresource else ""
        return f"Action({self.verb} {self.resource.plural}{sub} {self.namespace}/{self.name})"


Reactor = Callable[[Action], "tuple[bool, Any, BaseException | None]"]


class FakeClient(KubeClient):
    def __init__(self, state: ClusterState | None = None, *, cluster_name: str = "fake", simple: bool = True,
                 latency_s: float = 0.0):
        self.state = state or ClusterState(cluster_name, simple=simple)
        self.cluster_name = cluster_name
        self.actions: list[Action] = []
        self.reactors: list[tuple[str, str, Reactor]] = []
        self.latency_s = latency_s

    # -------------------------------------------------------------- test helpers
    def prepend_reactor(self, verb: str, resource: str, fn: Reactor) -> None:
        """`verb`/`resource` may be "*"; `fn` returns (handled, result, error)."""
        self.reactors.insert(0, (verb, resource, fn))

    def clear_actions(self) -> None:
        self.actions.clear()

    def writes(self, group: str | None = None) -> list[Action]:
        """Mutating actions, optionally only for one API group ("core" or the CRD group)."""
        out = [a for a in self.actions if a.verb not in ("get", "list", "watch")]
        return [a for a in out if group is None or a.group == group]

    def seed(self, rt: ResourceType, obj: dict) -> dict:
        """Preload an object without recording an action (NewSimpleClientset(objects...))."""
        ns = (obj.get("metadata") or {}).get("namespace", "")
        return self.state.create(rt, ns, obj)

    async def _record(self, a: Action):
        self.actions.append(a)
        if self.latency_s:
            await asyncio.sleep(self.latency_s)
        for verb, res, fn in self.reactors:
            if verb in ("*", a.verb) and res in ("*", a.resource.plural):
                handled, result, err = fn(a)
                if handled:
                    if err is not None:
                        raise err
                    return True, result
        return False, None

    # -------------------------------------------------------------- KubeClient
    async def get(self, rt, namespace, name):
        handled, res = await self._record(Action("get", rt, namespace, name))
        return res if handled else self.state.get(rt, namespace, name)

    async def list(self, rt, namespace, *, label_selector=None, limit=None, continue_token=None,
                   resource_version=None):
        handled, res = await self._record(Action("list", rt, namespace or ""))
        if handled:
            return res
        return self.state.list(rt, namespace, label_selector=label_selector, limit=limit,
                               continue_token=continue_token)

    async def create(self, rt, namespace, obj, *, field_manager=None):
        a = Action("create", rt, namespace, (obj.get("metadata") or {}).get("name", ""), obj=deep_copy(obj))
        handled, res = await self._record(a)
        return res if handled else self.state.create(rt, namespace, obj)

    async def update(self, rt, namespace, obj, *, field_manager=None):
        a = Action("update", rt, namespace, (obj.get("metadata") or {}).get("name", ""), obj=deep_copy(obj))
        handled, res = await self._record(a)
        return res if handled else self.state.update(rt, namespace, obj)

    async def update_status(self, rt, namespace, obj, *, field_manager=None):
        a = Action("update", rt, namespace, (obj.get("metadata") or {}).get("name", ""), subresource="status",
                   obj=deep_copy(obj))
        handled, res = await self._record(a)
        return res if handled else self.state.update(rt, namespace, obj, subresource="status")

    async def patch(self, rt, namespace, name, body, *, patch_type=PATCH_MERGE, field_manager=None, force=None,
                    subresource=None):
        a = Action("patch", rt, namespace, name, subresource=subresource or "", patch=deep_copy(body),
                   patch_type=patch_type)
        handled, res = await self._record(a)
        return res if handled else self.state.patch(rt, namespace, name, body, patch_type, subresource=subresource)

    async def delete(self, rt, namespace, name, *, propagation_policy=None, preconditions=None):
        handled, res = await self._record(Action("delete", rt, namespace, name))
        if handled:
            return res
        return self.state.delete(rt, namespace, name, preconditions=preconditions,
                                 propagation_policy=propagation_policy)

    async def watch(self, rt, namespace, *, resource_version=None, timeout_seconds=None, allow_bookmarks=True,
                    label_selector=None):
        handled, res = await self._record(Action("watch", rt, namespace or ""))
        if handled:
            return
        w = self.state.watch(rt, namespace, resource_version, label_selector)
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout_seconds if timeout_seconds else None
        try:
            while True:
                timeout = None if deadline is None else max(0.0, deadline - loop.time())
                try:
                    rec = await wait_timeout(w.queue.get(), timeout)
                except asyncio.TimeoutError:
                    return
                if rec is None:
                    return
                yield WatchEvent(rec.type, rec.obj)
        finally:
            w.close()
