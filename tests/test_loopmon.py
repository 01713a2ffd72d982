"""ncc/loopmon.py (event-loop stall monitor) and gctune's freeze loop."""
import asyncio
import gc
import json
import time

from ncc import gctune, loopmon


def test_monitor_off_without_env(monkeypatch):
    monkeypatch.delenv("NCC_LOOP_LAG_MS", raising=False)

    async def main():
        return loopmon.start("x")
    assert asyncio.run(main()) is None


def test_monitor_reports_blocked_loop_and_gc_pass(monkeypatch, tmp_path):
    path = tmp_path / "lag.jsonl"
    monkeypatch.setenv("NCC_LOOP_LAG_MS", "20")
    monkeypatch.setenv("NCC_LOOP_LAG_FILE", str(path))

    async def main():
        task = loopmon.start("unit")
        await asyncio.sleep(0.02)
        time.sleep(0.08)  # block the loop
        junk = [[i] for i in range(300_000)]  # noqa: F841 — a young generation worth scanning
        cb = gc.callbacks[-1]
        cb.threshold = 0.0  # report every GC pass
        gc.collect(0)
        await asyncio.sleep(0.02)
        task.cancel()
        await asyncio.gather(task, return_exceptions=True)
    n_callbacks = len(gc.callbacks)
    asyncio.run(main())
    assert len(gc.callbacks) == n_callbacks  # the GC hook is removed with the monitor
    rows = [json.loads(line) for line in path.read_text().splitlines()]
    stalls = [r for r in rows if "loop_lag_ms" in r]
    assert stalls and max(r["loop_lag_ms"] for r in stalls) >= 60 and stalls[0]["process"] == "unit"
    assert any(r.get("gc_pause_ms") is not None and r["generation"] == 0 for r in rows)


def test_freeze_loop_without_collect_only_freezes(monkeypatch):
    """The controllers' default freezes without a pass of its own; `collect=<generation>` runs that pass first
    and accounts for it in gctune.STATS."""
    calls = []
    monkeypatch.setattr(gctune.gc, "collect", lambda gen=2: calls.append(("collect", gen)) or 0)
    monkeypatch.setattr(gctune.gc, "freeze", lambda: calls.append(("freeze",)))

    async def main(**kw):
        t = asyncio.ensure_future(gctune.freeze_loop(0.01, **kw))
        await asyncio.sleep(0.035)
        t.cancel()
        await asyncio.gather(t, return_exceptions=True)
    asyncio.run(main())
    assert calls and all(c == ("freeze",) for c in calls)
    calls.clear()
    passes = gctune.STATS["passes"]
    asyncio.run(main(collect=1))
    assert ("collect", 1) in calls and ("freeze",) in calls and gctune.STATS["passes"] > passes
