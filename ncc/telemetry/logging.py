"""Structured logging (nexus-core `telemetry.ConfigureLogger` analogue).

stdout gets JSON (or text) records at the configured level (`log-level`, Helm
`controller.logLevel`).  When `DATADOG__API_KEY` and `DATADOG__ENDPOINT` are set
(deployment.yaml:70-95), records are also shipped to the Datadog HTTP intake in batches by a
background thread, tagged with `DATADOG__SERVICE_NAME` and `DATADOG__APPLICATION_HOST`, so a
slow or unreachable intake never blocks the event loop.
"""
from __future__ import annotations

import json
import logging
import os
import queue
import sys
import threading
import time
import urllib.request

_STD = set(logging.LogRecord("", 0, "", 0, "", (), None).__dict__) | {"message", "asctime"}

LEVELS = {"DEBUG": logging.DEBUG, "INFO": logging.INFO, "WARN": logging.WARNING, "WARNING": logging.WARNING,
          "ERROR": logging.ERROR, "FATAL": logging.CRITICAL, "CRITICAL": logging.CRITICAL}


def _record_dict(record: logging.LogRecord) -> dict:
    d = {"time": time.strftime("%Y-%m-%dT%H:%M:%S", time.gmtime(record.created)) + f".{int(record.msecs):03d}Z",
         "level": record.levelname, "logger": record.name, "msg": record.getMessage()}
    for k, v in record.__dict__.items():
        if k not in _STD and not k.startswith("_"):
            d[k] = v if isinstance(v, (str, int, float, bool, type(None))) else str(v)
    if record.exc_info:
        d["error"] = logging.Formatter().formatException(record.exc_info)
    return d


class JsonFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        return json.dumps(_record_dict(record))


class DatadogHandler(logging.Handler):
    """Batches records to the Datadog logs intake (v2 API) from a daemon thread."""

    def __init__(self, api_key: str, endpoint: str, service: str, host: str, batch: int = 100,
                 flush_interval: float = 2.0):
        super().__init__()
        site = endpoint if endpoint.startswith("http") else f"https://http-intake.logs.{endpoint}"
        self.url = site.rstrip("/") + "/api/v2/logs"
        self.api_key, self.service, self.host = api_key, service, host
        self.batch, self.flush_interval = batch, flush_interval
        self._q: queue.Queue = queue.Queue(maxsize=10000)
        self.dropped = 0
        threading.Thread(target=self._loop, name="ncc-datadog-logs", daemon=True).start()

    def emit(self, record: logging.LogRecord) -> None:
        d = _record_dict(record)
        d.update({"ddsource": "python", "service": self.service, "hostname": self.host, "status": record.levelname})
        try:
            self._q.put_nowait(d)
        except queue.Full:
            self.dropped += 1

    def _loop(self) -> None:
        while True:
            items = [self._q.get()]
            deadline = time.monotonic() + self.flush_interval
            while len(items) < self.batch and time.monotonic() < deadline:
                try:
                    items.append(self._q.get(timeout=max(0.0, deadline - time.monotonic())))
                except queue.Empty:
                    break
            try:
                req = urllib.request.Request(self.url, data=json.dumps(items).encode(), method="POST",
                                             headers={"Content-Type": "application/json", "DD-API-KEY": self.api_key})
                urllib.request.urlopen(req, timeout=5).read()
            except Exception:  # noqa: BLE001 — never let log shipping fail the process
                self.dropped += len(items)


def configure_logging(level: str = "INFO", fmt: str = "json", stream=None) -> logging.Logger:
    root = logging.getLogger()
    for h in list(root.handlers):
        root.removeHandler(h)
    h = logging.StreamHandler(stream or sys.stdout)
    h.setFormatter(JsonFormatter() if fmt == "json" else
                   logging.Formatter("%(asctime)s %(levelname)s %(name)s %(message)s"))
    root.addHandler(h)
    root.setLevel(LEVELS.get(str(level).upper(), logging.INFO))
    api_key, endpoint = os.environ.get("DATADOG__API_KEY"), os.environ.get("DATADOG__ENDPOINT")
    if api_key and endpoint:
        root.addHandler(DatadogHandler(api_key, endpoint,
                                       os.environ.get("DATADOG__SERVICE_NAME", "nexus-configuration-controller"),
                                       os.environ.get("DATADOG__APPLICATION_HOST", "")))
    # aiohttp's access/client loggers are chatty at DEBUG; keep them at WARNING.
    for noisy in ("aiohttp.access", "aiohttp.client", "aiohttp.internal", "asyncio"):
        logging.getLogger(noisy).setLevel(logging.WARNING)
    return root
