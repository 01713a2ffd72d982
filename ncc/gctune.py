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

THRESHOLDS = (50_000, 20, 100)


def tune(thresholds: tuple = THRESHOLDS) -> None:
    gc.set_threshold(*thresholds)
    gc.freeze()


async def freeze_loop(period: float = 5.0) -> None:
    """Collect young garbage, then freeze the survivors, every `period` seconds."""
    while True:
        await asyncio.sleep(period)
        gc.collect(1)
        gc.freeze()
