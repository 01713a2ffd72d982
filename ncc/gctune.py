"""Garbage-collector tuning for the long-running control-plane processes.

Cached Kubernetes objects are acyclic JSON dicts, so CPython's cyclic collector mostly re-scans live
caches: a full (gen-2) pass over a 30k-object store costs ~10-25 ms and lands at random points of a
propagation wave as a latency tail.  `tune()` raises the allocation thresholds and periodically moves
everything that survived into the permanent generation (`gc.freeze()`), so collections only look at
recent garbage.  Reference counting still frees objects immediately; only cycles created before a
freeze and later abandoned are kept (the asyncio machinery creates few, and they are short-lived).
"""
from __future__ import annotations

import asyncio
import gc
import time

THRESHOLDS = (50_000, 20, 100)
STATS = {"passes": 0, "collected": 0, "seconds": 0.0, "max_seconds": 0.0}  # freeze_loop's own passes


_auto = {"t0": 0.0}


def _on_gc(phase: str, info: dict) -> None:
    """Time every collection the interpreter runs (automatic ones included), per generation."""
    if phase == "start":
        _auto["t0"] = time.perf_counter()
        return
    dt = time.perf_counter() - _auto["t0"]
    g = info.get("generation", 0)
    STATS[f"gen{g}_n"] = STATS.get(f"gen{g}_n", 0) + 1
    STATS[f"gen{g}_s"] = round(STATS.get(f"gen{g}_s", 0.0) + dt, 4)
    STATS[f"gen{g}_max_s"] = round(max(STATS.get(f"gen{g}_max_s", 0.0), dt), 4)


def tune(thresholds: tuple = THRESHOLDS, account: bool = True) -> None:
    gc.set_threshold(*thresholds)
    gc.freeze()
    if account and _on_gc not in gc.callbacks:
        gc.callbacks.append(_on_gc)


async def freeze_loop(period: float = 1.0, collect: int | None = None) -> None:
    """Collect young garbage of generations up to `collect` (None: no pass of our own), then freeze the
    survivors, every `period` seconds.

    The controller processes default to freezing every second with no pass of their own: the automatic
    generation-0 collections (every 50 000 container allocations) still reclaim cycles that die young, and
    everything that survived one is frozen unscanned.  The round-2 policy, a generation-1 pass every 5 s,
    scans every young survivor: in the coordinator at 20 000 templates it found nothing to free in a whole
    run and stopped the loop for up to 250-300 ms each time; an explicit generation-0 pass every second
    found nothing either and cost 1.2 s of CPU per run (BENCHMARKS.md)."""
    while True:
        await asyncio.sleep(period)
        if collect is not None:
            t0 = time.perf_counter()
            STATS["collected"] += gc.collect(collect)
            dt = time.perf_counter() - t0
            STATS["passes"] += 1
            STATS["seconds"] += dt
            STATS["max_seconds"] = max(STATS["max_seconds"], dt)
        gc.freeze()
