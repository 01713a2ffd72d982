"""The cluster-client interface every transport implements.

The reference holds two typed clientsets per cluster (client-go `kubernetes.Interface` for
CoreV1 and the nexus-core clientset for ScienceV1 — main.go:58-68).  This
framework uses ONE generic client per cluster parameterised by `ResourceType`; per-API-group
behaviour (rate limiting, action logs in tests) is keyed on `ResourceType.group_key`.

Implementations:
  * `ncc.kube.rest.RestClient`         — aiohttp over HTTP(S) against a real/fake apiserver
  * `ncc.testing.fake_client.FakeClient` — in-memory, records actions (client-go fake analogue)
  * `RateLimitedClient` (below)         — decorator adding client-go's per-group token bucket
"""
from __future__ import annotations

import abc
from typing import AsyncIterator, NamedTuple

from ..api.resources import ResourceType
from .ratelimit import AsyncRateLimiter

PATCH_MERGE = "application/merge-patch+json"
PATCH_STRATEGIC = "application/strategic-merge-patch+json"
PATCH_JSON = "application/json-patch+json"
PATCH_APPLY = "application/apply-patch+yaml"


class WatchEvent(NamedTuple):
    type: str  # ADDED | MODIFIED | DELETED | BOOKMARK | ERROR
    object: dict


class KubeClient(abc.ABC):
    """Async client for one cluster."""

    cluster_name: str = ""

    @abc.abstractmethod
    async def get(self, rt: ResourceType, namespace: str, name: str) -> dict: ...

    @abc.abstractmethod
    async def list(self, rt: ResourceType, namespace: str | None, *, label_selector: str | None = None,
                   limit: int | None = None, continue_token: str | None = None,
                   resource_version: str | None = None) -> dict: ...

    @abc.abstractmethod
    async def create(self, rt: ResourceType, namespace: str, obj: dict, *, field_manager: str | None = None) -> dict: ...

    @abc.abstractmethod
    async def update(self, rt: ResourceType, namespace: str, obj: dict, *, field_manager: str | None = None) -> dict: ...

    @abc.abstractmethod
    async def update_status(self, rt: ResourceType, namespace: str, obj: dict, *,
                            field_manager: str | None = None) -> dict: ...

    @abc.abstractmethod
    async def patch(self, rt: ResourceType, namespace: str, name: str, body, *, patch_type: str = PATCH_MERGE,
                    field_manager: str | None = None, force: bool | None = None,
                    subresource: str | None = None) -> dict: ...

    @abc.abstractmethod
    async def delete(self, rt: ResourceType, namespace: str, name: str, *, propagation_policy: str | None = None,
                     preconditions: dict | None = None) -> dict | None: ...

    @abc.abstractmethod
    def watch(self, rt: ResourceType, namespace: str | None, *, resource_version: str | None = None,
              timeout_seconds: int | None = None, allow_bookmarks: bool = True,
              label_selector: str | None = None) -> AsyncIterator[WatchEvent]: ...

    async def close(self) -> None:  # pragma: no cover - default no-op
        return None


class RateLimitedClient(KubeClient):
    """Wraps a client with one token bucket per API group (client-go RESTClient semantics).

    Watches take a token when the stream is opened, as a client-go watch request does.
    """

    def __init__(self, inner: KubeClient, qps: float, burst: int):
        self.inner = inner
        self.cluster_name = inner.cluster_name
        self.qps, self.burst = qps, burst
        self._limiters: dict[str, AsyncRateLimiter] = {}

    def limiter(self, rt: ResourceType) -> AsyncRateLimiter:
        lim = self._limiters.get(rt.group_key)
        if lim is None:
            lim = self._limiters[rt.group_key] = AsyncRateLimiter(self.qps, self.burst)
        return lim

    def throttled_seconds(self) -> float:
        return sum(l.waited_s for l in self._limiters.values())

    async def get(self, rt, namespace, name):
        await self.limiter(rt).wait()
        return await self.inner.get(rt, namespace, name)

    async def list(self, rt, namespace, **kw):
        await self.limiter(rt).wait()
        return await self.inner.list(rt, namespace, **kw)

    async def create(self, rt, namespace, obj, **kw):
        await self.limiter(rt).wait()
        return await self.inner.create(rt, namespace, obj, **kw)

    async def update(self, rt, namespace, obj, **kw):
        await self.limiter(rt).wait()
        return await self.inner.update(rt, namespace, obj, **kw)

    async def update_status(self, rt, namespace, obj, **kw):
        await self.limiter(rt).wait()
        return await self.inner.update_status(rt, namespace, obj, **kw)

    async def patch(self, rt, namespace, name, body, **kw):
        await self.limiter(rt).wait()
        return await self.inner.patch(rt, namespace, name, body, **kw)

    @property
    def write_meta(self):
        """Rate-limited pass-through of the inner client's `write_meta`, or None when it has none."""
        inner = getattr(self.inner, "write_meta", None)
        if inner is None:
            return None

        async def wm(verb, rt, namespace, body, **kw):
            await self.limiter(rt).wait()
            return await inner(verb, rt, namespace, body, **kw)
        return wm

    async def delete(self, rt, namespace, name, **kw):
        await self.limiter(rt).wait()
        return await self.inner.delete(rt, namespace, name, **kw)

    async def watch(self, rt, namespace, **kw):
        await self.limiter(rt).wait()
        async for ev in self.inner.watch(rt, namespace, **kw):
            yield ev

    def __getattr__(self, name):
        """The inner client's extensions: raw watch streams (the watch relay's — a token per stream opened,
        as `watch`), and anything else read-only (`stats`, `supports_line_tap`, ...)."""
        inner = getattr(self.inner, name)  # AttributeError when the inner client has none (hasattr → False)
        if name in ("watch_raw", "watch_raw_batches"):
            async def raw(rt, namespace, **kw):
                await self.limiter(rt).wait()
                async for x in inner(rt, namespace, **kw):
                    yield x
            return raw
        return inner

    async def close(self):
        await self.inner.close()
