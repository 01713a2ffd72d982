"""asyncio helpers.

`wait_timeout` replaces `asyncio.wait_for`: on Python 3.10 `wait_for` can swallow a cancellation
that races with the inner awaitable completing (bpo-42130), which leaves a "cancelled" task
running forever — exactly what a controller's shutdown path cannot afford.  `asyncio.wait`
never swallows the caller's cancellation; the inner task is cancelled explicitly.
"""
from __future__ import annotations

import asyncio


def _retrieve(fut: asyncio.Future) -> None:
    """Mark the outcome of an abandoned future as seen (a cancelled gather() finishes with a CancelledError
    *exception*, which asyncio would otherwise log as never retrieved)."""
    if not fut.cancelled():
        fut.exception()


def _abandon(task: asyncio.Future) -> None:
    task.cancel()
    task.add_done_callback(_retrieve)


async def wait_timeout(aw, timeout: float | None):
    """Await `aw` with a timeout (raises asyncio.TimeoutError); cancellation-safe."""
    task = asyncio.ensure_future(aw)
    if timeout is None:
        try:
            return await task
        except asyncio.CancelledError:
            _abandon(task)
            raise
    try:
        done, _ = await asyncio.wait({task}, timeout=timeout)
    except asyncio.CancelledError:
        _abandon(task)
        raise
    if not done:
        _abandon(task)
        raise asyncio.TimeoutError()
    return task.result()
