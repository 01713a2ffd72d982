"""Work queue semantics (client-go workqueue parity) for the Python core, the C++ core, and the asyncio facade."""
import asyncio

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from ncc import native
from ncc.workqueue.core import (BucketRateLimiter, ItemExponentialFailureRateLimiter, MaxOfRateLimiter,
                                PyRateLimitingQueue)
from ncc.workqueue.queue import WorkQueue

NATIVE = native.load()
CORES = [("py", lambda *a: PyRateLimitingQueue(*a))]
if NATIVE is not None:
    CORES.append(("native", lambda *a: NATIVE.RateLimitingQueue(*a)))


@pytest.fixture(params=[c[0] for c in CORES])
def make(request):
    return dict(CORES)[request.param]


def test_dedup_and_fifo(make):
    q = make(0.01, 1.0, 10.0, 100)
    assert q.add("a") and q.add("b") and not q.add("a")
    assert q.length() == 2
    assert q.try_get() == "a" and q.try_get() == "b" and q.try_get() is None


def test_busy_covers_queued_processing_and_waiting(make):
    q = make(0.01, 1.0, 10.0, 10)
    assert not q.busy("a")
    q.add("a")
    assert q.busy("a")
    assert q.try_get() == "a"
    assert q.busy("a")  # processing
    q.done("a")
    assert not q.busy("a")
    q.add_after("b", 0.5, 0.0)
    assert q.busy("b")  # waiting for its delayed add
    assert q.promote(1.0) == 1 and q.busy("b")


def test_exclusive_processing_requeues_on_done(make):
    q = make(0.01, 1.0, 10.0, 100)
    q.add("a")
    assert q.try_get() == "a"
    assert not q.add("a")          # parked: "a" is being processed
    assert q.try_get() is None     # never handed to a second worker
    assert q.done("a")             # dirty → re-queued
    assert q.try_get() == "a"
    assert not q.done("a")


def test_delays_earliest_ready_wins(make):
    q = make(0.01, 1.0, 10.0, 100)
    q.add_after("a", 5.0, 100.0)
    q.add_after("a", 1.0, 100.0)   # earlier ready time replaces the later one
    q.add_after("a", 3.0, 100.0)   # later one ignored
    assert q.next_ready_in(100.0) == pytest.approx(1.0)
    assert q.promote(100.5) == 0
    assert q.promote(101.0) == 1
    assert q.try_get() == "a"
    assert q.promote(200.0) == 0   # superseded heap entries are dropped
    assert q.next_ready_in(200.0) == -1.0


def test_exponential_backoff_and_forget(make):
    q = make(0.03, 5.0, 0.0, 1)   # qps 0 disables the bucket
    delays = [q.add_rate_limited("k", 0.0) for _ in range(10)]
    assert delays[:4] == pytest.approx([0.03, 0.06, 0.12, 0.24])
    assert max(delays) == 5.0 and q.num_requeues("k") == 10
    q.forget("k")
    assert q.num_requeues("k") == 0
    assert q.add_rate_limited("k", 0.0) == pytest.approx(0.03)


def test_bucket_limits_retry_storms(make):
    q = make(0.0001, 0.0001, 10.0, 2)
    d = [q.add_rate_limited(f"k{i}", 0.0) for i in range(5)]
    assert d[0] == 0.0001 and d[1] == 0.0001       # within burst: per-item backoff dominates
    assert d[2] == pytest.approx(0.1) and d[3] == pytest.approx(0.2) and d[4] == pytest.approx(0.3)


def test_shutdown_rejects_adds(make):
    q = make(0.01, 1.0, 10.0, 100)
    q.shutdown()
    assert q.shutting_down() and not q.add("x") and q.length() == 0


def test_limiters_match_client_go():
    e = ItemExponentialFailureRateLimiter(0.005, 1000.0)
    assert [e.when("x", 0) for _ in range(3)] == [0.005, 0.01, 0.02]
    b = BucketRateLimiter(1.0, 1)
    assert b.when("x", 0.0) == 0.0 and b.when("y", 0.0) == pytest.approx(1.0) and b.when("z", 0.5) == pytest.approx(1.5)
    m = MaxOfRateLimiter(ItemExponentialFailureRateLimiter(0.5, 10.0), BucketRateLimiter(100.0, 10))
    assert m.when("x", 0.0) == 0.5 and m.num_requeues("x") == 1


ops = st.lists(st.tuples(st.sampled_from(["add", "get", "done", "after", "limited", "forget", "promote", "tick"]),
                         st.sampled_from(["a", "b", "c", "d"]),
                         st.floats(min_value=0.0, max_value=0.5)), max_size=120)


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
@settings(max_examples=300, deadline=None)
@given(ops)
def test_native_matches_python_reference(seq):
    """Same op sequence + same clock → identical observable results (C++ core ≡ Python reference)."""
    py = PyRateLimitingQueue(0.01, 0.2, 20.0, 3)
    nat = NATIVE.RateLimitingQueue(0.01, 0.2, 20.0, 3)
    now = 0.0
    held: list[str] = []
    for op, key, x in seq:
        if op == "tick":
            now += x
            continue
        if op == "add":
            r = (py.add(key), nat.add(key))
        elif op == "get":
            r = (py.try_get(), nat.try_get())
            if r[0] is not None:
                held.append(r[0])
        elif op == "done":
            k = held.pop(0) if held else key
            r = (py.done(k), nat.done(k))
        elif op == "after":
            r = (py.add_after(key, x, now), nat.add_after(key, x, now))
        elif op == "limited":
            r = (py.add_rate_limited(key, now), nat.add_rate_limited(key, now))
            assert r[0] == pytest.approx(r[1])
            r = (None, None)
        elif op == "forget":
            r = (py.forget(key), nat.forget(key))
        else:
            r = (py.promote(now), nat.promote(now))
        assert r[0] == r[1], (op, key, r)
        assert py.length() == nat.length()
        assert py.num_requeues(key) == nat.num_requeues(key)
        assert py.next_ready_in(now) == pytest.approx(nat.next_ready_in(now))
        assert all(py.busy(k) == nat.busy(k) for k in "abcd")


@pytest.mark.parametrize("native_core", [False] + ([True] if NATIVE is not None else []))
async def test_async_facade_workers_and_delays(native_core):
    q = WorkQueue(base_delay=0.01, max_delay=0.05, qps=100.0, burst=10, native=native_core)
    assert q.is_native == native_core
    seen = []
    active = set()

    async def worker():
        while True:
            k = await q.get()
            if k is None:
                return
            assert k not in active  # exclusive processing across workers
            active.add(k)
            seen.append(k)
            await asyncio.sleep(0.001)
            active.discard(k)
            q.done(k)

    ws = [asyncio.ensure_future(worker()) for _ in range(4)]
    for i in range(20):
        q.add(f"k{i % 5}")
    q.add_after("late", 0.05)
    q.add_rate_limited("retry")
    await asyncio.sleep(0.2)
    assert "late" in seen and "retry" in seen
    assert {f"k{i}" for i in range(5)} <= set(seen)
    q.shutdown()
    await asyncio.wait_for(asyncio.gather(*ws), 2)
