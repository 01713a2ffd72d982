"""DogStatsD metrics client (nexus-core `telemetry.WithStatsd/Gauge/GaugeDuration` analogue).

The reference emits `nexus_configuration_controller.reconcile_latency` and
`.workqueue_length` gauges per processed item (controller.go:50-56,389-390; main.go:44).
The sink address comes from `DD_DOGSTATSD_URL` (`udp://host:port` or `unix:///path`, Helm
default `unix:///var/run/datadog/dsd.socket`, values.yaml:190-192), falling back to
`DD_AGENT_HOST`/`DD_DOGSTATSD_PORT`.  Unified-service tags come from `DD_SERVICE`,
`DD_VERSION`, `DD_ENV` and origin detection from `DD_ENTITY_ID` (deployment.yaml:85-95).

Sends are fire-and-forget datagrams on a non-blocking socket, aggregated client-side and
flushed once a second: a missing agent never slows the reconcile loop.  `MemoryMetrics`
records values for tests; `MultiMetrics` fans out (e.g. to the optional Prometheus exporter).
"""
from __future__ import annotations

import asyncio
import os
import socket
import time
from collections import defaultdict


class Metrics:
    def gauge(self, name: str, value: float, tags: dict | None = None, rate: float = 1.0) -> None: ...

    def gauge_duration(self, name: str, start: float, tags: dict | None = None, rate: float = 1.0) -> None:
        """Gauge of the elapsed milliseconds since `start` (a time.monotonic() value)."""
        self.gauge(name, (time.monotonic() - start) * 1000.0, tags, rate)

    def count(self, name: str, value: float = 1, tags: dict | None = None, rate: float = 1.0) -> None: ...

    def histogram(self, name: str, value: float, tags: dict | None = None, rate: float = 1.0) -> None: ...

    def close(self) -> None: ...


class NullMetrics(Metrics):
    def gauge(self, name, value, tags=None, rate=1.0):
        return None

    def count(self, name, value=1, tags=None, rate=1.0):
        return None

    def histogram(self, name, value, tags=None, rate=1.0):
        return None


class MemoryMetrics(Metrics):
    def __init__(self):
        self.values: dict[str, list[float]] = defaultdict(list)

    def gauge(self, name, value, tags=None, rate=1.0):
        self.values[name].append(float(value))

    def count(self, name, value=1, tags=None, rate=1.0):
        self.values[name].append(float(value))

    def histogram(self, name, value, tags=None, rate=1.0):
        self.values[name].append(float(value))


class MultiMetrics(Metrics):
    def __init__(self, *sinks: Metrics):
        self.sinks = [s for s in sinks if s is not None]

    def gauge(self, name, value, tags=None, rate=1.0):
        for s in self.sinks:
            s.gauge(name, value, tags, rate)

    def count(self, name, value=1, tags=None, rate=1.0):
        for s in self.sinks:
            s.count(name, value, tags, rate)

    def histogram(self, name, value, tags=None, rate=1.0):
        for s in self.sinks:
            s.histogram(name, value, tags, rate)

    def close(self):
        for s in self.sinks:
            s.close()


def _format_tags(tags: dict | None, constant: list[str]) -> str:
    items = list(constant)
    if tags:
        items.extend(f"{k}:{v}" if v not in (None, "") else str(k) for k, v in tags.items())
    return "|#" + ",".join(items) if items else ""


class StatsdClient(Metrics):
    """DogStatsD over UDP/UDS with client-side aggregation, like datadog-go v5's default client.

    Gauges keep the last value and counts are summed per (name, tags) within a flush interval;
    histograms are buffered.  Everything goes out as newline-joined packets (≤ `max_packet` bytes)
    from a loop timer, so a reconcile costs a dict update instead of a syscall."""

    def __init__(self, namespace: str, url: str | None = None, constant_tags: list[str] | None = None,
                 flush_interval: float = 1.0, max_packet: int = 1432, aggregate: bool = True):
        self.namespace = namespace.rstrip(".") + "." if namespace else ""
        self.url = url or default_url()
        self.constant_tags = list(constant_tags if constant_tags is not None else default_tags())
        self.flush_interval = flush_interval
        self.max_packet = max_packet
        self.aggregate = aggregate
        self.sent = 0
        self.dropped = 0
        self._sock = None
        self._addr = None
        self._gauges: dict = {}
        self._counts: dict = {}
        self._lines: list[str] = []
        self._timer = None
        self._open()

    def _open(self) -> None:
        url = self.url
        try:
            if url.startswith("unix://"):
                path = url[len("unix://"):]
                s = socket.socket(socket.AF_UNIX, socket.SOCK_DGRAM)
                self._addr = path
            else:
                hostport = url[len("udp://"):] if url.startswith("udp://") else url
                host, _, port = hostport.rpartition(":")
                host = host.strip("[]") or "127.0.0.1"
                fam = socket.AF_INET6 if ":" in host else socket.AF_INET
                s = socket.socket(fam, socket.SOCK_DGRAM)
                self._addr = (host, int(port or 8125))
            s.setblocking(False)
            self._sock = s
        except (OSError, ValueError):
            self._sock = None

    def _send(self, payload: str) -> None:
        if self._sock is None:
            self.dropped += 1
            return
        try:
            self._sock.sendto(payload.encode(), self._addr)
            self.sent += 1
        except OSError:
            self.dropped += 1

    def _line(self, name: str, value: float, kind: str, tags, rate: float) -> str:
        sr = f"|@{rate}" if rate < 1.0 else ""
        t = dict(tags) if tags and not isinstance(tags, dict) else tags
        return f"{self.namespace}{name}:{value:g}|{kind}{sr}{_format_tags(t, self.constant_tags)}"

    def _schedule(self) -> None:
        if self._timer is not None:
            return
        try:
            loop = asyncio.get_running_loop()
        except RuntimeError:
            return  # no running loop: buffered until flush()/close()
        self._timer = loop.call_later(self.flush_interval, self.flush)

    def flush(self) -> None:
        self._timer = None
        lines = self._lines
        self._lines = []
        for (name, tags), v in self._gauges.items():
            lines.append(self._line(name, v, "g", tags, 1.0))
        for (name, tags), v in self._counts.items():
            lines.append(self._line(name, v, "c", tags, 1.0))
        self._gauges.clear()
        self._counts.clear()
        buf: list[str] = []
        size = 0
        for ln in lines:
            if buf and size + len(ln) + 1 > self.max_packet:
                self._send("\n".join(buf))
                buf, size = [], 0
            buf.append(ln)
            size += len(ln) + 1
        if buf:
            self._send("\n".join(buf))

    @staticmethod
    def _key(name, tags):
        return name, (tuple(sorted(tags.items())) if tags else None)

    def gauge(self, name, value, tags=None, rate=1.0):
        if not self.aggregate:
            self._send(self._line(name, value, "g", tags, rate))
            return
        self._gauges[self._key(name, tags)] = value
        self._schedule()

    def count(self, name, value=1, tags=None, rate=1.0):
        if not self.aggregate:
            self._send(self._line(name, value, "c", tags, rate))
            return
        k = self._key(name, tags)
        self._counts[k] = self._counts.get(k, 0) + value
        self._schedule()

    def histogram(self, name, value, tags=None, rate=1.0):
        if not self.aggregate:
            self._send(self._line(name, value, "h", tags, rate))
            return
        self._lines.append(self._line(name, value, "h", tags, rate))
        self._schedule()

    def close(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        self.flush()
        if self._sock is not None:
            self._sock.close()
            self._sock = None


def default_url() -> str:
    url = os.environ.get("DD_DOGSTATSD_URL")
    if url:
        return url
    host = os.environ.get("DD_AGENT_HOST", "127.0.0.1")
    port = os.environ.get("DD_DOGSTATSD_PORT", "8125")
    return f"udp://{host}:{port}"


def default_tags() -> list[str]:
    tags = []
    for env, tag in (("DD_SERVICE", "service"), ("DD_VERSION", "version"), ("DD_ENV", "env")):
        v = os.environ.get(env)
        if v:
            tags.append(f"{tag}:{v}")
    ent = os.environ.get("DD_ENTITY_ID")
    if ent:
        tags.append(f"dd.internal.entity_id:{ent}")
    return tags
