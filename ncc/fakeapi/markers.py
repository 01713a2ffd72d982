"""Server-side propagation probes for benchmarks.

A marker is a field path per resource (e.g. `nexusalgorithmtemplates=spec.container.versionTag`,
`secrets=data.version`).  On every committed write the server extracts the marker value and
records the wall-clock commit time (`time.time_ns()`) the first time each object reaches each
value.  A benchmark writes a wave of changes with a new marker value into the controller
cluster and then asks each shard server to wait until N objects carry it; the recorded commit
times give exact controller→shard propagation latencies without any client-side watch
(which would itself load the shard apiserver and blur the measurement).
"""
from __future__ import annotations

import asyncio
import time

from ..aio import wait_timeout


def _extract(obj: dict, path: list[str]):
    cur = obj
    for p in path:
        if not isinstance(cur, dict):
            return None
        cur = cur.get(p)
        if cur is None:
            return None
    return cur if isinstance(cur, (str, int, float)) else None


class MarkerTracker:
    def __init__(self, specs: dict[str, str] | None = None):
        self.paths = {plural: path.split(".") for plural, path in (specs or {}).items()}
        self.first_seen: dict[tuple, dict] = {}  # (plural, value) -> {name: t_ns}
        self._waiters: list[tuple[list, asyncio.Future]] = []
        self._thresholds: dict[tuple, set] = {}  # (plural, value) -> counts some waiter needs

    def add_spec(self, plural: str, path: str) -> None:
        self.paths[plural] = path.split(".")

    def on_write(self, type_: str, rt, obj: dict) -> None:
        if type_ == "DELETED":
            return
        path = self.paths.get(rt.plural)
        if path is None:
            return
        v = _extract(obj, path)
        if v is None:
            return
        m = obj.get("metadata") or {}
        bk = (rt.plural, str(v))
        bucket = self.first_seen.get(bk)
        if bucket is None:
            bucket = self.first_seen[bk] = {}
        key = f"{m.get('namespace', '')}/{m.get('name', '')}"
        if key not in bucket:
            bucket[key] = time.time_ns()
            # re-evaluate waiters only when this write completes one of their counts
            if self._waiters and len(bucket) in self._thresholds.get(bk, ()):
                self._check()

    def satisfied(self, want: list) -> bool:
        return all(len(self.first_seen.get((w["plural"], str(w["value"])), ())) >= int(w["count"]) for w in want)

    def _check(self) -> None:
        keep = []
        for want, fut in self._waiters:
            if fut.done():
                continue
            if self.satisfied(want):
                fut.set_result(True)
            else:
                keep.append((want, fut))
        self._waiters = keep
        if not keep:
            self._thresholds.clear()

    async def wait(self, want: list, timeout: float) -> bool:
        if self.satisfied(want):
            return True
        fut = asyncio.get_running_loop().create_future()
        self._waiters.append((want, fut))
        for w in want:
            self._thresholds.setdefault((w["plural"], str(w["value"])), set()).add(int(w["count"]))
        try:
            return await wait_timeout(fut, timeout)
        except asyncio.TimeoutError:
            return False

    def times(self, plural: str, value, keyed: bool = False):
        """Commit times of objects that reached `value`: a list, or {"ns/name": t_ns} when keyed."""
        b = self.first_seen.get((plural, str(value)), {})
        return dict(b) if keyed else list(b.values())

    def counts(self) -> dict:
        return {f"{p}={v}": len(b) for (p, v), b in self.first_seen.items()}
