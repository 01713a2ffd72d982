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


def test_freeze_loop_policies(monkeypatch):
    """The controllers' default: every tick a freeze becomes due, performed at the end of the next
    generation-1 collection (young generations empty: cycles abandoned by failing passes are not frozen
    unscanned), or by a generation-1 pass of our own when none ran within a tick; every `full_period` an
    unfreeze + full collection.  `young=False` (the fake apiservers) only freezes; `collect=<generation>`
    always runs that pass first.  Each pass is accounted in gctune.STATS."""
    calls = []
    monkeypatch.setattr(gctune.gc, "collect", lambda gen=2: calls.append(("collect", gen)) or 0)
    monkeypatch.setattr(gctune.gc, "freeze", lambda: calls.append(("freeze",)))
    monkeypatch.setattr(gctune.gc, "unfreeze", lambda: calls.append(("unfreeze",)))
    monkeypatch.setattr(gctune.gc, "get_freeze_count", lambda: 0)
    monkeypatch.setitem(gctune._auto, "freeze_due", False)

    async def main(until, **kw):
        # run the loop until `until()` holds (at most 5 s): a loaded host may give it fewer ticks than the
        # wall clock would — waiting a fixed 35 ms made this test flaky under a parallel suite
        t = asyncio.ensure_future(gctune.freeze_loop(0.01, **kw))
        loop = asyncio.get_running_loop()
        end = loop.time() + 5.0
        await asyncio.sleep(0.035)
        while not until() and loop.time() < end:
            await asyncio.sleep(0.01)
        t.cancel()
        await asyncio.gather(t, return_exceptions=True)
    asyncio.run(main(lambda: bool(calls), young=False, full_period=0))
    assert calls and all(c == ("freeze",) for c in calls)
    calls.clear()
    young = gctune.STATS["young_n"]
    # quiet process: no collection ran, so a generation-1 pass of ours (an automatic generation-1 collection
    # in between makes the tick leave the freeze to it instead: the test's own gc hooks are mocked out, so
    # keep the interpreter's collector from running meanwhile)
    gctune.gc.disable()
    try:
        asyncio.run(main(lambda: len(calls) >= 2, full_period=0))
    finally:
        gctune.gc.enable()
    assert calls[:2] == [("collect", 1), ("freeze",)] and ("unfreeze",) not in calls
    assert gctune.STATS["young_n"] > young
    calls.clear()
    # a generation-1 collection ran since the last tick: the freeze is left due, for the next one to perform
    gctune._auto["freeze_due"] = False
    seen = gctune._auto["gen1_runs"]
    gctune._auto["gen1_runs"] += 1
    assert gctune.young_then_freeze(seen) == seen + 1 and calls == [] and gctune._auto["freeze_due"]
    gctune._on_gc("start", {"generation": 0})
    gctune._on_gc("stop", {"generation": 0})  # a generation-0 pass leaves generation 1 as it was: no freeze
    assert calls == [] and gctune._auto["freeze_due"]
    gctune._on_gc("start", {"generation": 1})
    gctune._on_gc("stop", {"generation": 1})
    assert calls == [("freeze",)] and not gctune._auto["freeze_due"]
    calls.clear()
    full = gctune.STATS["full_n"]
    asyncio.run(main(lambda: ("unfreeze",) in calls, full_period=0.015, idle=lambda: True))
    assert ("unfreeze",) in calls and ("collect", 2) in calls and gctune.STATS["full_n"] > full
    calls.clear()
    # busy: the full collection waits for an idle moment, at most another period
    assert not gctune.full_due(0.9, 1.0, lambda: True)
    assert gctune.full_due(1.0, 1.0, lambda: True) and gctune.full_due(1.0, 1.0, None)
    assert not gctune.full_due(1.5, 1.0, lambda: False) and gctune.full_due(2.0, 1.0, lambda: False)
    passes = gctune.STATS["passes"]
    asyncio.run(main(lambda: ("collect", 1) in calls and ("freeze",) in calls, collect=1, full_period=0))
    assert ("collect", 1) in calls and ("freeze",) in calls and gctune.STATS["passes"] > passes
