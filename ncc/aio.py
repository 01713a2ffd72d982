"""asyncio helpers.

`wait_timeout` replaces `asyncio.wait_for`: on Python 3.10 `wait_for` can swallow a cancellation
that races with the inner awaitable completing (bpo-42130), which leaves a "cancelled" task
running forever — exactly what a controller's shutdown path cannot afford.  `asyncio.wait`
never swallows the caller's cancellation; the inner task is cancelled explicitly.
"""
from __future__ import annotations

import asyncio


async def wait_timeout(aw, timeout: float | None):
    """Await `aw` with a timeout (raises asyncio.TimeoutError); cancellation-safe."""
    task = asyncio.ensure_future(aw)
    if timeout is None:
        return await task
    try:
        done, _ = await asyncio.wait({task}, timeout=timeout)
    except asyncio.CancelledError:
        task.cancel()
        raise
    if not done:
        task.cancel()
        raise asyncio.TimeoutError()
    return task.result()
