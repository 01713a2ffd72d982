"""Lease-based leader election (`coordination.k8s.io/v1` Lease), for running more than one replica.

The reference supports a single replica only: its Helm chart pins `replicas: 1` with the
`Recreate` strategy ("NCC only supports single replica", .helm/templates/deployment.yaml:15-19)
and there is no leader election (SURVEY.md §5.3 "HA: none").  With `leader-elect: true` this
framework runs N replicas: one holds the Lease and reconciles, the others wait as warm standbys —
controller and shard informers listed and watching, shard executors spawned with their caches
synced, only the reconcile workers gated (`App.run`) — and take over within `lease-duration` of
the leader dying, or immediately when the leader releases the Lease on a clean shutdown.

Semantics follow the usual Kubernetes controller pattern:
* expiry is judged on the *local* clock from when this candidate last saw the Lease record change
  (holder / renewTime), never by comparing wall clocks across machines;
* every acquire/renew is an optimistic-concurrency PUT (resourceVersion), so two candidates can
  never both win — the loser gets 409 and keeps waiting;
* the leader renews every `retry-period`, each attempt bounded by the rest of the renew deadline; if
  it cannot renew for `renew-deadline` it stops leading: workers are cancelled and executors killed at
  once (no draining writes), and the app exits non-zero so its replacement starts from a clean slate;
* release on shutdown empties `holderIdentity` so a standby takes over without waiting.
"""
from __future__ import annotations

import asyncio
import logging
import os
import random
import socket
import time
import uuid
from datetime import datetime, timezone

from .api import resources as R
from .kube import errors as E
from .kube.client import KubeClient

log = logging.getLogger("ncc.leader")


def micro_now() -> str:
    """metav1.MicroTime wire format."""
    return datetime.now(timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def default_identity() -> str:
    return f"{socket.gethostname()}_{uuid.uuid4()}"


class LeaderElector:
    def __init__(self, client: KubeClient, namespace: str, name: str, identity: str | None = None, *,
                 lease_duration: float = 15.0, renew_deadline: float = 10.0, retry_period: float = 2.0,
                 clock=time.monotonic):
        if not lease_duration > renew_deadline > retry_period > 0:
            raise ValueError("leader election needs lease-duration > renew-deadline > retry-period > 0")
        self.client = client
        self.namespace = namespace
        self.name = name
        self.identity = identity or default_identity()
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.clock = clock
        self.leading = False
        self.transitions = 0
        self._observed_key = None
        self._observed_at = 0.0
        self._lease: dict | None = None

    # ------------------------------------------------------------------ one attempt
    def _observe(self, spec: dict) -> None:
        key = (spec.get("holderIdentity"), spec.get("renewTime"), spec.get("leaseDurationSeconds"))
        if key != self._observed_key:
            self._observed_key = key
            self._observed_at = self.clock()

    def _spec(self, prev: dict | None) -> dict:
        now = micro_now()
        prev = prev or {}
        spec = dict(prev)
        if prev.get("holderIdentity") != self.identity:
            spec["acquireTime"] = now
            spec["leaseTransitions"] = int(prev.get("leaseTransitions") or 0) + (1 if prev else 0)
        spec.update(holderIdentity=self.identity, leaseDurationSeconds=max(1, int(round(self.lease_duration))),
                    renewTime=now)
        return spec

    async def try_acquire_or_renew(self) -> bool:
        """One round trip pair: read the Lease, take or renew it if allowed.  Never raises for API errors."""
        try:
            try:
                cur = await self.client.get(R.LEASES, self.namespace, self.name)
            except E.NotFound:
                body = {"apiVersion": R.LEASES.api_version, "kind": R.LEASES.kind,
                        "metadata": {"name": self.name, "namespace": self.namespace}, "spec": self._spec(None)}
                res = await self.client.create(R.LEASES, self.namespace, body)
                return self._won(res)
            spec = cur.get("spec") or {}
            self._observe(spec)
            holder = spec.get("holderIdentity") or ""
            duration = float(spec.get("leaseDurationSeconds") or self.lease_duration)
            if holder and holder != self.identity and self._observed_at + duration > self.clock():
                self.leading = False
                return False  # held by someone else and not (yet) expired
            upd = dict(cur)
            upd["spec"] = self._spec(spec)
            res = await self.client.update(R.LEASES, self.namespace, upd)
            return self._won(res)
        except (E.Conflict, E.AlreadyExists):
            return False  # lost the race; re-read next round
        except (E.ApiError, OSError, asyncio.TimeoutError) as e:
            log.warning("lease %s/%s: %s", self.namespace, self.name, e)
            return False

    def _won(self, lease: dict) -> bool:
        if not self.leading:
            self.transitions += 1
            log.info("acquired lease %s/%s as %s", self.namespace, self.name, self.identity)
        self.leading = True
        self._lease = lease
        self._observe(lease.get("spec") or {})
        return True

    # ------------------------------------------------------------------ loops
    async def _sleep(self, seconds: float, stop: asyncio.Event | None) -> bool:
        """Sleep, waking early when `stop` is set; returns True if stopped."""
        if stop is None:
            await asyncio.sleep(seconds)
            return False
        if stop.is_set():
            return True
        waiter = asyncio.ensure_future(stop.wait())
        try:
            await asyncio.wait([waiter], timeout=seconds)
        finally:
            if not waiter.done():
                waiter.cancel()
        return stop.is_set()

    async def acquire(self, stop: asyncio.Event | None = None) -> bool:
        """Block until this candidate leads (True) or `stop` is set (False)."""
        waited = False
        while True:
            if await self.try_acquire_or_renew():
                return True
            if not waited:
                log.info("waiting for lease %s/%s (held by %s)", self.namespace, self.name,
                         (self._observed_key or ("?",))[0])
                waited = True
            if await self._sleep(self.retry_period * (1.0 + 0.2 * random.random()), stop):
                return False

    async def hold(self, stop: asyncio.Event | None = None, on_lost=None) -> None:
        """Renew every `retry_period` until `stop`; give up after `renew_deadline` without a renewal.

        Each renew attempt is itself bounded by what is left of the renew deadline (client-go bounds it
        with RenewDeadline the same way): a renew stuck in a slow request or Retry-After back-off must not
        outlive the deadline, or a standby could take the expired Lease while this replica still writes."""
        last_ok = self.clock()
        while True:
            if await self._sleep(self.retry_period, stop):
                return
            budget = self.renew_deadline - (self.clock() - last_ok)
            ok = False
            if budget > 0:
                try:
                    ok = await asyncio.wait_for(self.try_acquire_or_renew(), timeout=budget)
                except asyncio.TimeoutError:
                    log.warning("lease %s/%s: renew did not finish within the renew deadline", self.namespace,
                                self.name)
            if ok:
                last_ok = self.clock()
                continue
            if not self.leading or self.clock() - last_ok >= self.renew_deadline:
                self.leading = False
                log.error("lost lease %s/%s", self.namespace, self.name)
                if on_lost is not None:
                    on_lost()
                return

    async def release(self) -> bool:
        """Give the Lease up (empty holder, 1 s duration) so a standby can take over at once."""
        if not self.leading or self._lease is None:
            return False
        self.leading = False
        try:
            cur = await self.client.get(R.LEASES, self.namespace, self.name)
            spec = dict(cur.get("spec") or {})
            if spec.get("holderIdentity") != self.identity:
                return False
            spec.update(holderIdentity="", leaseDurationSeconds=1, renewTime=micro_now())
            upd = dict(cur)
            upd["spec"] = spec
            await self.client.update(R.LEASES, self.namespace, upd)
            log.info("released lease %s/%s", self.namespace, self.name)
            return True
        except (E.ApiError, OSError, asyncio.TimeoutError) as e:
            log.warning("releasing lease %s/%s: %s", self.namespace, self.name, e)
            return False


def identity_from_env() -> str:
    """POD_NAME (downward API) when present, else hostname + random suffix."""
    pod = os.environ.get("POD_NAME")
    return f"{pod}_{uuid.uuid4().hex[:8]}" if pod else default_identity()
