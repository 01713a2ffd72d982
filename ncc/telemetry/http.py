"""Optional HTTP endpoints: Prometheus `/metrics`, `/healthz`, `/readyz`.

The reference exposes neither (its Deployment has no probes); these are
framework additions enabled by `metrics-bind-address` / `health-bind-address`.
"""
from __future__ import annotations

from typing import Callable

from aiohttp import web

from .statsd import Metrics

try:
    import prometheus_client as prom
except ImportError:  # pragma: no cover
    prom = None


class PrometheusMetrics(Metrics):
    """Mirrors every statsd gauge into a Prometheus gauge/histogram in a private registry."""

    def __init__(self, namespace: str):
        if prom is None:
            raise RuntimeError("prometheus_client not installed")
        self.namespace = namespace
        self.registry = prom.CollectorRegistry()
        self._gauges: dict = {}
        self._counters: dict = {}
        self._hists: dict = {}

    def _labels(self, tags):
        return tuple(sorted((tags or {}).keys()))

    def gauge(self, name, value, tags=None, rate=1.0):
        key = (name, self._labels(tags))
        g = self._gauges.get(key)
        if g is None:
            g = self._gauges[key] = prom.Gauge(name, name, list(key[1]), namespace=self.namespace,
                                               registry=self.registry)
        (g.labels(**tags) if tags else g).set(value)

    def count(self, name, value=1, tags=None, rate=1.0):
        key = (name, self._labels(tags))
        c = self._counters.get(key)
        if c is None:
            c = self._counters[key] = prom.Counter(name, name, list(key[1]), namespace=self.namespace,
                                                   registry=self.registry)
        (c.labels(**tags) if tags else c).inc(value)

    def histogram(self, name, value, tags=None, rate=1.0):
        key = (name, self._labels(tags))
        h = self._hists.get(key)
        if h is None:
            h = self._hists[key] = prom.Histogram(name, name, list(key[1]), namespace=self.namespace,
                                                  registry=self.registry)
        (h.labels(**tags) if tags else h).observe(value)

    def render(self) -> bytes:
        return prom.generate_latest(self.registry)


def _split(addr: str) -> tuple[str, int]:
    host, _, port = addr.rpartition(":")
    return (host or "0.0.0.0"), int(port)


class OpsServer:
    def __init__(self, ready: Callable[[], bool], prometheus: PrometheusMetrics | None = None,
                 extra: Callable[[], dict] | None = None, checks: Callable[[], list] | None = None):
        """`checks()` → [(name, ok, detail)]: what `/readyz?verbose` lists, as the kube-apiserver's does."""
        self.ready = ready
        self.prometheus = prometheus
        self.extra = extra
        self.checks = checks
        self.app = web.Application()
        self.app.router.add_get("/healthz", self._healthz)
        self.app.router.add_get("/readyz", self._readyz)
        self.app.router.add_get("/metrics", self._metrics)
        self.app.router.add_get("/debug/state", self._state)
        self._runner = None
        self.port = None

    async def _healthz(self, _r):
        return web.Response(text="ok")

    async def _readyz(self, r):
        ready = self.ready()
        if "verbose" not in r.query:
            return web.Response(text="ok") if ready else web.Response(status=503, text="not ready")
        lines = [f"[{'+' if ok else '-'}]{name} {detail}".rstrip() for name, ok, detail in
                 (self.checks() if self.checks else [])]
        lines.append("readyz check passed" if ready else "readyz check failed")
        return web.Response(status=200 if ready else 503, text="\n".join(lines) + "\n")

    async def _metrics(self, _r):
        if self.prometheus is None:
            return web.Response(status=404, text="metrics disabled")
        return web.Response(body=self.prometheus.render(), content_type="text/plain")

    async def _state(self, _r):
        return web.json_response(self.extra() if self.extra else {})

    async def start(self, addr: str) -> int:
        host, port = _split(addr)
        self._runner = web.AppRunner(self.app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, host, port)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
        return self.port

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
