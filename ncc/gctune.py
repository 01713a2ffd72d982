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


async def freeze_loop(period: float = 5.0, collect: bool = True) -> None:
    """Collect young garbage, then freeze the survivors, every `period` seconds.

    `collect=False` freezes without the generation-1 pass.  That pass scans every young survivor, and in a
    process that retains most of what it allocates (the fake apiserver's store and watch history: ~1M
    containers in 5 s at bench rates) it found nothing to free and stopped the loop for 130-240 ms.
    Freezing instead keeps the cycles that died after surviving a generation-0 pass."""
    while True:
        await asyncio.sleep(period)
        if collect:
            gc.collect(1)
        gc.freeze()
