"""Event correlator semantics, and the multi-rank benchmark path over gloo (world_size 2, CPU)."""
import asyncio
import json
import os
import socket
import subprocess
import sys

import pytest

from ncc.api import resources as R
from ncc.controller.events import SPAM_BURST, BroadcastRecorder, FakeRecorder
from ncc.fakeapi.storage import ClusterState
from ncc.testing.fake_client import FakeClient
from ncc.testing.workload import make_template

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


async def _drain(rec):
    await asyncio.wait_for(asyncio.gather(*(q.join() for q in rec._queues)), 5)


async def test_event_dedup_patches_count():
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False)
    rec.start()
    t = client.state.create(R.TEMPLATES, "nexus", make_template(0, "nexus"))
    for _ in range(3):
        rec.event(t, "Normal", "Synced", "Resource of type NexusAlgorithmTemplate synced successfully")
    await _drain(rec)
    events = client.state.list(R.EVENTS, "nexus")["items"]
    assert len(events) == 1 and events[0]["count"] == 3 and events[0]["involvedObject"]["kind"] == "NexusAlgorithmTemplate"
    assert events[0]["source"]["component"] == "nexus-configuration-controller"
    assert rec.stats["created"] == 1 and rec.stats["patched"] == 2
    await rec.stop()


async def test_event_coalescing_folds_pending_repeats():
    """Native mode: repeats of an event still waiting for its writer ride on that write (count + n); the
    Event object ends up exactly as with one write per occurrence."""
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False, writers=4, coalesce=True)
    t = client.state.create(R.TEMPLATES, "nexus", make_template(0, "nexus"))
    other = client.state.create(R.TEMPLATES, "nexus", make_template(1, "nexus"))
    msg = "Resource of type NexusAlgorithmTemplate synced successfully"
    for _ in range(3):
        rec.event(t, "Normal", "Synced", msg)
    rec.event(other, "Normal", "Synced", msg)
    rec.event(t, "Warning", "ErrResourceSyncError", "boom")  # a different event is not folded
    rec.start()
    await _drain(rec)
    rec.event(t, "Normal", "Synced", msg)  # written already: a repeat PATCHes the count
    await _drain(rec)
    events = {(e["involvedObject"]["name"], e["reason"]): e for e in client.state.list(R.EVENTS, "nexus")["items"]}
    assert events[(t["metadata"]["name"], "Synced")]["count"] == 4
    assert events[(other["metadata"]["name"], "Synced")]["count"] == 1
    assert events[(t["metadata"]["name"], "ErrResourceSyncError")]["count"] == 1
    assert rec.stats["merged"] == 2 and rec.stats["created"] == 3 and rec.stats["patched"] == 1
    assert not rec._pending
    await rec.stop()


async def test_event_spam_filter_and_aggregation():
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False)
    rec.start()
    t = client.state.create(R.TEMPLATES, "nexus", make_template(0, "nexus"))
    for i in range(SPAM_BURST + 10):
        rec.event(t, "Warning", "ErrResourceSyncError", f"failure #{i}")
    await _drain(rec)
    assert rec.stats["dropped_spam"] == 10
    msgs = [e["message"] for e in client.state.list(R.EVENTS, "nexus")["items"]]
    assert any(m.startswith("(combined from similar events)") for m in msgs)
    # distinct messages beyond the aggregation threshold collapse into one aggregate event
    assert len(msgs) <= 10
    await rec.stop()


async def test_event_spam_fast_drop_lets_the_next_token_through(monkeypatch):
    """An object whose spam bucket is empty is dropped on a fast path until its next token is due (1/300 s
    refill): the event after that is written, and one more is dropped again — the bucket's own verdicts."""
    from ncc.controller import events as ev
    clock = [1000.0]
    monkeypatch.setattr(ev.time, "monotonic", lambda: clock[0])
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False)
    t = client.state.create(R.TEMPLATES, "nexus", make_template(0, "nexus"))
    other = client.state.create(R.TEMPLATES, "nexus", make_template(1, "nexus"))
    for _ in range(SPAM_BURST + 5):
        rec.event(t, "Normal", "Synced", "synced")
    assert rec.stats["dropped_spam"] == 5 and len(rec._blocked) == 1
    rec.event(other, "Normal", "Synced", "synced")  # another object is not held back
    assert rec.stats["dropped_spam"] == 5
    clock[0] += 299.0
    rec.event(t, "Normal", "Synced", "synced")
    assert rec.stats["dropped_spam"] == 6
    clock[0] += 1.5
    rec.event(t, "Normal", "Synced", "synced")
    rec.event(t, "Normal", "Synced", "synced")
    assert rec.stats["dropped_spam"] == 7 and rec.stats["recorded"] == SPAM_BURST + 9


async def test_event_writers_keep_per_object_order():
    """Several writer tasks: each object's events stay on one writer, so dedup PATCHes count correctly."""
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False, writers=4)
    rec.start()
    ts = [client.state.create(R.TEMPLATES, "nexus", make_template(i, "nexus")) for i in range(12)]
    for _ in range(5):
        for t in ts:
            rec.event(t, "Normal", "Synced", "Resource of type NexusAlgorithmTemplate synced successfully")
    await _drain(rec)
    events = client.state.list(R.EVENTS, "nexus")["items"]
    assert len(events) == 12 and all(e["count"] == 5 for e in events)
    assert rec.stats["created"] == 12 and rec.stats["patched"] == 48
    assert sum(1 for q in rec._queues if q.qsize() == 0) == 4
    await rec.stop()


async def test_event_correlator_caches_are_bounded():
    """client-go keeps its correlator state in 4096-entry LRUs; so do we (no growth with object count)."""
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False, writers=4)
    rec.start()
    for i in range(5000):
        rec.event({"kind": "NexusAlgorithmTemplate", "apiVersion": "science.sneaksanddata.com/v1",
                   "metadata": {"name": f"t{i}", "namespace": "nexus", "uid": f"u{i}"}},
                  "Normal", "Synced", "synced")
        if i % 500 == 499:
            await _drain(rec)
    await _drain(rec)
    assert rec.stats["created"] == 5000
    for cache in (rec._buckets, rec._similar, rec._seen):
        assert 0 < len(cache) <= 4096
    await rec.stop()


async def test_native_correlator_cache_follows_the_object_count():
    """Native mode sizes the correlator caches to the objects managed (a callable limit): with 5000 objects
    emitting events, each object's repeat is still a count PATCH of its first Event, not a new Event."""
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False, writers=4, cache_limit=lambda: 2 * 5000)
    rec.start()

    def obj(i):
        return {"kind": "NexusAlgorithmTemplate", "apiVersion": "science.sneaksanddata.com/v1",
                "metadata": {"name": f"t{i}", "namespace": "nexus", "uid": f"u{i}"}}
    for rnd in range(2):
        for i in range(5000):
            rec.event(obj(i), "Normal", "Synced", "synced")
            if i % 500 == 499:
                await _drain(rec)
        await _drain(rec)
    assert rec.stats["created"] == 5000 and rec.stats["patched"] == 5000
    assert len(rec._seen) == 5000
    await rec.stop()


async def test_warning_is_held_not_dropped_when_the_buffer_is_full():
    """Native mode: a flood of `Synced` Events fills the writers' buffer (client-go drops past it, and so do
    we for Normal events), but a Warning recorded meanwhile is held and written once there is room."""
    client = FakeClient(ClusterState(), simple=False)
    gate = asyncio.Event()
    real_create = client.create

    async def slow_create(rt, ns, body, **kw):
        await gate.wait()
        return await real_create(rt, ns, body, **kw)
    client.create = slow_create
    rec = BroadcastRecorder(client, log_events=False, writers=1, coalesce=True, repeat_window=1.0)
    rec._write_meta = None  # through client.create
    rec.start()

    def obj(i):
        return {"kind": "NexusAlgorithmTemplate", "apiVersion": "science.sneaksanddata.com/v1",
                "metadata": {"name": f"t{i}", "namespace": "nexus", "uid": f"u{i}"}}
    for i in range(1100):  # one blocked in the writer, 1000 buffered, the rest dropped
        rec.event(obj(i), "Normal", "Synced", "synced")
        await asyncio.sleep(0) if i == 0 else None
    assert rec.stats["dropped_full"] > 0
    rec.event(obj(5000), "Warning", "ErrResourceExists", "Secret already exists")
    assert rec.stats["warnings_held"] == 1
    gate.set()
    for _ in range(500):
        if any(e["reason"] == "ErrResourceExists" for e in client.state.list(R.EVENTS, "nexus")["items"]):
            break
        await asyncio.sleep(0.01)
    assert any(e["reason"] == "ErrResourceExists" for e in client.state.list(R.EVENTS, "nexus")["items"])
    await rec.stop()


def test_fake_recorder_formats_like_client_go():
    r = FakeRecorder()
    r.event({}, "Warning", "ErrResourceMissing", "msg")
    assert r.events == ["Warning ErrResourceMissing msg"]
    silent = FakeRecorder(keep=False)
    silent.event({}, "Normal", "Synced", "x")
    assert silent.events == []


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_bench_two_ranks_over_gloo():
    """The driver's N>1 launch shape: torch.distributed.run, one shard apiserver per rank, rank 0 reports — with
    the TLS + product-defaults second run the driver's command includes (both runs share the process group)."""
    pytest.importorskip("torch.distributed")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--templates", "40", "--steps", "2", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["shards"] == 2 and res["scaling"] == "weak"
    assert res["value"] > 0 and res["p50_latency_ms"] is not None and res["controller_alive"]
    assert res["tls_value"] > 0 and res["tls_config"]["controller_transport"] == "h2"


@pytest.mark.slow
def test_bench_eight_ranks_auto_sized_topology():
    """The driver's N=8 launch on a large host, rehearsed here: NCC_CPU_SHARE=128 makes the automatic
    sizing pick what it would on an 8-GPU node with ≥128 CPUs (ncc/app.py `auto_sizing`: native executors,
    k=1 per shard, C=2 coordinator partitions (one per 4 shards) sharing the executors → 1 partition child +
    8 executors under the controller).
    Every wave must converge with no process restarted and the controller alive."""
    pytest.importorskip("torch.distributed")
    from ncc.app import auto_sizing
    from ncc.controller.native_executor import binary_path
    native = binary_path() is not None
    k, c = auto_sizing(8, cpus=128, native=native)
    env = dict(os.environ, NCC_CPU_SHARE="128")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "8", "--templates", "40", "--steps", "2", "--warmup", "1", "--timeout", "120",
           "--no-tls-run"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 8 and res["config"]["shards"] == 8 and res["controller_alive"]
    sz = res["controller_sizing"]
    # the C coordinators share the parent's k executors per shard
    assert sz["cpus"] == 128 and sz["coordinator_partitions"] == c and sz["executors_per_shard"] == k
    assert sz["executor_impl"] == ("native" if native else "python")
    want_children = (c - 1) + 8 * k
    ch = res["controller_children"]
    assert ch == {"start": want_children, "end": want_children, "replaced": 0}, (ch, sz)
    assert res["value"] > 0 and res["p50_latency_ms"] is not None
    print(json.dumps(res))


async def test_event_repeat_window_folds_repeats_of_written_events():
    """Native mode `event-repeat-window`: the first occurrence is written at once; repeats of an Event already
    written are held for the window and go out as one count PATCH — the Event ends up with the same count."""
    client = FakeClient(ClusterState(), simple=False)
    rec = BroadcastRecorder(client, log_events=False, writers=4, coalesce=True, repeat_window=0.05)
    rec.start()
    t = client.state.create(R.TEMPLATES, "nexus", make_template(0, "nexus"))
    msg = "Resource of type NexusAlgorithmTemplate synced successfully"
    rec.event(t, "Normal", "Synced", msg)
    await _drain(rec)
    assert rec.stats["created"] == 1
    for _ in range(5):  # repeats within one window
        rec.event(t, "Normal", "Synced", msg)
    rec.event(t, "Warning", "ErrResourceSyncError", "boom")  # a new event is not held
    await _drain(rec)
    assert rec.stats["patched"] == 0 and rec.stats["created"] == 2
    await asyncio.sleep(0.1)
    await _drain(rec)
    events = {e["reason"]: e for e in client.state.list(R.EVENTS, "nexus")["items"]}
    assert events["Synced"]["count"] == 6 and rec.stats["patched"] == 1
    # many held repeats are never dropped for a full writer buffer
    ts = [client.state.create(R.TEMPLATES, "nexus", make_template(i, "nexus")) for i in range(1, 1600)]
    for k in range(0, len(ts), 200):  # first occurrences, at a pace the writers keep up with
        for o in ts[k:k + 200]:
            rec.event(o, "Normal", "Synced", msg)
        await _drain(rec)
    assert rec.stats["dropped_full"] == 0
    for o in ts:  # then one burst of repeats: more than the writers' buffers hold
        rec.event(o, "Normal", "Synced", msg)
    await asyncio.sleep(0.5)
    await _drain(rec)
    await rec.stop()
    counts = [e["count"] for e in client.state.list(R.EVENTS, "nexus")["items"] if e["reason"] == "Synced"]
    assert len(counts) == 1600 and sorted(counts)[:1599] == [2] * 1599, rec.stats
    assert rec.stats["dropped_full"] == 0
