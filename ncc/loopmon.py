"""Event-loop stall monitor for the Python processes (coordinator, Python executors, fake apiservers).

`NCC_LOOP_LAG_MS=<threshold>` starts a coroutine that sleeps 2 ms at a time and records every wake-up
that came more than `threshold` ms late: the loop was blocked (a long callback, a GC pass, the process
descheduled).  Each stall, and each GC pass longer than the threshold, is one JSON line — process, wall-clock end of the stall, its length, and the
cyclic-GC time spent inside it — appended to `NCC_LOOP_LAG_FILE` (default: stderr).  The wall clock is
`time.time_ns()`, the clock the fake apiservers stamp commits with, so stalls line up with a bench wave's
per-object timings.  `NCC_LOOP_LAG_DEBUG=1` also runs the loop in asyncio debug mode (slower) and writes
asyncio's "Executing <callback> took N seconds" reports past the threshold, which name the callback.
"""
from __future__ import annotations

import asyncio
import gc
import json
import logging
import os
import sys
import time

PERIOD = 0.002


class _GcClock:
    """Total time in cyclic-GC passes; a pass longer than the threshold is reported on its own."""
    def __init__(self, name: str, threshold_ms: float, out):
        self.total = 0.0
        self._t0 = 0.0
        self.name, self.threshold, self.out = name, threshold_ms, out

    def __call__(self, phase: str, info: dict) -> None:
        if phase == "start":
            self._t0 = time.perf_counter()
            return
        dt = time.perf_counter() - self._t0
        self.total += dt
        if dt * 1e3 > self.threshold:
            self.out.write(json.dumps({"gc_pause_ms": round(dt * 1e3, 2), "process": self.name,
                                       "generation": info.get("generation"), "collected": info.get("collected"),
                                       "end_ns": time.time_ns()}) + "\n")


class _JsonLines(logging.Handler):
    def __init__(self, name: str, out):
        super().__init__(logging.WARNING)
        self.name_, self.out = name, out

    def emit(self, record: logging.LogRecord) -> None:
        self.out.write(json.dumps({"asyncio": record.getMessage()[:500], "process": self.name_,
                                   "end_ns": time.time_ns()}) + "\n")


async def _monitor(name: str, threshold_ms: float, path: str | None) -> None:
    out = open(path, "a", buffering=1) if path else sys.stderr
    gcc = _GcClock(name, threshold_ms, out)
    gc.callbacks.append(gcc)
    handler = None
    if os.environ.get("NCC_LOOP_LAG_DEBUG") == "1":
        loop = asyncio.get_running_loop()
        loop.set_debug(True)
        loop.slow_callback_duration = threshold_ms / 1e3
        handler = _JsonLines(name, out)
        logging.getLogger("asyncio").addHandler(handler)
    try:
        last, gc_last = time.perf_counter(), 0.0
        while True:
            await asyncio.sleep(PERIOD)
            now = time.perf_counter()
            lag = (now - last - PERIOD) * 1e3
            if lag > threshold_ms:
                out.write(json.dumps({"loop_lag_ms": round(lag, 2), "process": name, "pid": os.getpid(),
                                      "end_ns": time.time_ns(),
                                      "gc_ms": round((gcc.total - gc_last) * 1e3, 2)}) + "\n")
            last, gc_last = now, gcc.total
    finally:
        gc.callbacks.remove(gcc)
        if handler is not None:
            logging.getLogger("asyncio").removeHandler(handler)
        if path:
            out.close()


def start(name: str) -> asyncio.Future | None:
    """Start the monitor in the running loop when NCC_LOOP_LAG_MS is set; returns its task (or None)."""
    thr = os.environ.get("NCC_LOOP_LAG_MS")
    if not thr:
        return None
    return asyncio.ensure_future(_monitor(name, float(thr), os.environ.get("NCC_LOOP_LAG_FILE") or None))
