"""Fake kube-apiserver fidelity: the substrate every integration test and benchmark stands on."""
import asyncio

import pytest

from ncc.api import resources as R
from ncc.fakeapi.server import FakeApiServer
from ncc.fakeapi.storage import ClusterState
from ncc.kube import errors as E
from ncc.kube.client import PATCH_APPLY, PATCH_JSON, PATCH_MERGE, PATCH_STRATEGIC
from ncc.kube.kubeconfig import ClusterConfig
from ncc.kube.rest import RestClient
from ncc.testing.workload import make_configmap, make_secret, make_template

NS = "nexus"


def test_create_assigns_metadata_and_rejects_duplicates():
    s = ClusterState()
    o = s.create(R.TEMPLATES, NS, make_template(1, NS))
    m = o["metadata"]
    assert m["uid"] and m["resourceVersion"] == "1" and m["generation"] == 1 and m["creationTimestamp"]
    with pytest.raises(E.AlreadyExists):
        s.create(R.TEMPLATES, NS, make_template(1, NS))
    bad = make_template(2, NS)
    bad["metadata"]["resourceVersion"] = "5"
    with pytest.raises(E.BadRequest):
        s.create(R.TEMPLATES, NS, bad)


def test_update_conflicts_noops_generation_and_status_isolation():
    s = ClusterState()
    o = s.create(R.TEMPLATES, NS, make_template(1, NS))
    stale = dict(o, metadata=dict(o["metadata"]))
    o2 = s.update(R.TEMPLATES, NS, dict(o, spec=dict(o["spec"], command="bash")))
    assert o2["metadata"]["generation"] == 2 and o2["metadata"]["resourceVersion"] == "2"
    with pytest.raises(E.Conflict):
        s.update(R.TEMPLATES, NS, stale)
    same = s.update(R.TEMPLATES, NS, o2)   # no-op: no RV bump, no event
    assert same["metadata"]["resourceVersion"] == "2" and s.stats["noop_update"] == 1
    st = s.update(R.TEMPLATES, NS, dict(o2, status={"conditions": [{"type": "Ready"}]}), subresource="status")
    assert st["metadata"]["generation"] == 2 and st["status"]["conditions"][0]["type"] == "Ready"
    # a main-resource write cannot change status
    back = s.update(R.TEMPLATES, NS, dict(st, status={}, spec=dict(st["spec"], command="sh")))
    assert back["status"] == st["status"] and back["metadata"]["generation"] == 3


def test_gc_deletes_orphans_and_strips_dangling_refs():
    s = ClusterState()
    t1 = s.create(R.TEMPLATES, NS, make_template(1, NS))
    t2 = s.create(R.TEMPLATES, NS, make_template(2, NS))
    ref = lambda t: {"apiVersion": "science.sneaksanddata.com/v1", "kind": "NexusAlgorithmTemplate",  # noqa: E731
                     "name": t["metadata"]["name"], "uid": t["metadata"]["uid"]}
    only = make_secret("only", NS)
    only["metadata"]["ownerReferences"] = [ref(t1)]
    shared = make_configmap("shared", NS)
    shared["metadata"]["ownerReferences"] = [ref(t1), ref(t2)]
    s.create(R.SECRETS, NS, only)
    s.create(R.CONFIGMAPS, NS, shared)
    s.delete(R.TEMPLATES, NS, t1["metadata"]["name"])
    with pytest.raises(E.NotFound):
        s.get(R.SECRETS, NS, "only")
    left = s.get(R.CONFIGMAPS, NS, "shared")
    assert [r["uid"] for r in left["metadata"]["ownerReferences"]] == [t2["metadata"]["uid"]]


async def test_watch_replay_and_gone():
    s = ClusterState(history=3)
    s.create(R.SECRETS, NS, make_secret("a", NS))      # rv1
    w = s.watch(R.SECRETS, NS, "1")
    s.create(R.SECRETS, NS, make_secret("b", NS))      # rv2
    s.delete(R.SECRETS, NS, "a")                       # rv3
    evs = [await w.queue.get(), await w.queue.get()]
    assert [e.type for e in evs] == ["ADDED", "DELETED"] and evs[1].obj["metadata"]["resourceVersion"] == "3"
    for i in range(5):
        s.create(R.SECRETS, NS, make_secret(f"x{i}", NS))
    with pytest.raises(E.Gone):
        s.watch(R.SECRETS, NS, "1")
    w0 = s.watch(R.SECRETS, NS, "0")                    # synthetic ADDED for current objects
    assert w0.queue.qsize() == 6


def test_patches():
    s = ClusterState()
    s.create(R.CONFIGMAPS, NS, make_configmap("c", NS))
    o = s.patch(R.CONFIGMAPS, NS, "c", {"data": {"k": "v", "version": None}}, PATCH_MERGE)
    assert o["data"]["k"] == "v" and "version" not in o["data"]
    o = s.patch(R.CONFIGMAPS, NS, "c", [{"op": "replace", "path": "/data/k", "value": "w"}], PATCH_JSON)
    assert o["data"]["k"] == "w"
    o = s.patch(R.CONFIGMAPS, NS, "c", {"metadata": {"ownerReferences": [{"uid": "u1", "name": "t"}]}},
                PATCH_STRATEGIC)
    o = s.patch(R.CONFIGMAPS, NS, "c", {"metadata": {"ownerReferences": [{"uid": "u2", "name": "t2"}]}},
                PATCH_STRATEGIC)
    assert [r["uid"] for r in o["metadata"]["ownerReferences"]] == ["u1", "u2"]
    a = s.patch(R.SECRETS, NS, "applied", {"apiVersion": "v1", "kind": "Secret", "data": {"x": "eQ=="}}, PATCH_APPLY)
    assert a["metadata"]["uid"] and a["data"] == {"x": "eQ=="}


def test_list_pagination_and_selectors():
    s = ClusterState()
    for i in range(7):
        sec = make_secret(f"s{i}", NS)
        sec["metadata"]["labels"] = {"tier": "gpu" if i % 2 else "cpu"}
        s.create(R.SECRETS, NS, sec)
    page = s.list(R.SECRETS, NS, limit=3)
    names = [o["metadata"]["name"] for o in page["items"]]
    while page["metadata"].get("continue"):
        page = s.list(R.SECRETS, NS, limit=3, continue_token=page["metadata"]["continue"])
        names += [o["metadata"]["name"] for o in page["items"]]
    assert names == [f"s{i}" for i in range(7)]
    assert len(s.list(R.SECRETS, NS, label_selector="tier=gpu")["items"]) == 3
    assert len(s.list(R.SECRETS, NS, label_selector="tier in (gpu,cpu),tier!=cpu")["items"]) == 3


@pytest.mark.parametrize("transport", ["fast", "aiohttp"])
async def test_http_roundtrip_watch_bookmarks_auth_and_faults(transport):
    srv = FakeApiServer(name="t", token="sekret", bookmark_interval=0.05)
    url = await srv.start()
    good = RestClient(ClusterConfig(server=url, token="sekret"), transport=transport)
    bad = RestClient(ClusterConfig(server=url, token="nope"), transport=transport)
    try:
        with pytest.raises(E.Unauthorized):
            await bad.list(R.SECRETS, NS)
        created = await good.create(R.TEMPLATES, NS, make_template(0, NS))
        got = await good.get(R.TEMPLATES, NS, created["metadata"]["name"])
        assert got == created
        with pytest.raises(E.NotFound):
            await good.get(R.TEMPLATES, NS, "missing")
        with pytest.raises(E.AlreadyExists):
            await good.create(R.TEMPLATES, NS, make_template(0, NS))
        lst = await good.list(R.TEMPLATES, NS)
        rv = lst["metadata"]["resourceVersion"]
        events = []

        async def consume():
            async for ev in good.watch(R.TEMPLATES, NS, resource_version=rv, timeout_seconds=1):
                events.append(ev.type)
                if ev.type == "MODIFIED":
                    return
        task = asyncio.ensure_future(consume())
        await asyncio.sleep(0.15)
        upd = dict(got, spec=dict(got["spec"], command="bash"))
        await good.update(R.TEMPLATES, NS, upd)
        await asyncio.wait_for(task, 3)
        assert "BOOKMARK" in events and events[-1] == "MODIFIED"
        st = await good.update_status(R.TEMPLATES, NS, dict(await good.get(R.TEMPLATES, NS, "algo-00000"),
                                                             status={"syncedToClusters": ["a"]}))
        assert st["status"]["syncedToClusters"] == ["a"]
        srv.faults.update({"error_rate": 1.0, "error_code": 500})
        with pytest.raises(E.InternalError):
            await good.create(R.SECRETS, NS, make_secret("s", NS))
        srv.faults.update({"error_rate": 0.0, "down": True})
        with pytest.raises(E.ServiceUnavailable):
            await good.list(R.SECRETS, NS)
        srv.faults.update({"down": False})
        await good.delete(R.TEMPLATES, NS, "algo-00000")
        with pytest.raises(E.NotFound):
            await good.delete(R.TEMPLATES, NS, "algo-00000")
    finally:
        await good.close()
        await bad.close()
        await srv.stop()


async def test_http_gone_is_reported_in_stream():
    srv = FakeApiServer(state=ClusterState(history=2))
    url = await srv.start()
    c = RestClient(ClusterConfig(server=url))
    try:
        for i in range(5):
            await c.create(R.SECRETS, NS, make_secret(f"s{i}", NS))
        evs = [ev async for ev in c.watch(R.SECRETS, NS, resource_version="1", timeout_seconds=1)]
        assert evs[0].type == "ERROR" and evs[0].object["code"] == 410
    finally:
        await c.close()
        await srv.stop()


async def test_transport_survives_server_side_close():
    """A keep-alive connection the server closed is retried once on a fresh connection."""
    srv = FakeApiServer()
    url = await srv.start()
    c = RestClient(ClusterConfig(server=url), transport="fast")
    try:
        await c.create(R.SECRETS, NS, make_secret("a", NS))
        for conn in list(srv._http._conns):
            conn.transport.close()
        await asyncio.sleep(0.05)
        assert (await c.get(R.SECRETS, NS, "a"))["metadata"]["name"] == "a"
    finally:
        await c.close()
        await srv.stop()


async def test_pipelined_transport_orders_responses_and_recovers():
    """pipeline_depth > 1: with both pool connections busy, further requests are pipelined; responses are
    matched in order (errors included), and a connection the server drops fails over to a fresh one."""
    srv = FakeApiServer()
    url = await srv.start()
    c = RestClient(ClusterConfig(server=url), transport="fast", pool_size=2, pipeline_depth=16)
    try:
        res = await asyncio.gather(*(c.create(R.SECRETS, NS, make_secret(f"s{i}", NS)) for i in range(40)))
        assert [r["metadata"]["name"] for r in res] == [f"s{i}" for i in range(40)]
        pool = c._pool
        assert pool.opened <= 2 and srv.state.count(R.SECRETS, NS) == 40
        # interleaved successes and errors on the same pipelined connections stay matched
        jobs = []
        for i in range(40):
            jobs.append(c.get(R.SECRETS, NS, f"s{i}" if i % 2 == 0 else f"missing{i}"))
        out = await asyncio.gather(*jobs, return_exceptions=True)
        for i, r in enumerate(out):
            if i % 2 == 0:
                assert r["metadata"]["name"] == f"s{i}"
            else:
                assert isinstance(r, E.NotFound)
        for conn in list(srv._http._conns):
            conn.transport.close()
        await asyncio.sleep(0.05)
        got = await asyncio.gather(*(c.get(R.SECRETS, NS, f"s{i}") for i in range(10)))
        assert [g["metadata"]["name"] for g in got] == [f"s{i}" for i in range(10)]
    finally:
        await c.close()
        await srv.stop()


async def test_control_endpoints_stage_apply_markers_and_seeding():
    """The load generator's control plane (bench.py, bench/suite.py drive it from other processes): marker
    probes, staged and direct applies, seeding of owned dependents, admission/fault switches and stats."""
    import aiohttp
    srv = FakeApiServer(name="ctl")
    url = await srv.start()
    try:
        async with aiohttp.ClientSession() as s:
            async def post(what, body):
                async with s.post(f"{url}/_fake/{what}", json=body) as r:
                    return r.status, await r.json()
            st, out = await post("markers", {"specs": {"secrets": "data.version"}})
            assert st == 200 and out["specs"]["secrets"] == "data.version"
            sec = make_secret("m0", NS, version=1)
            st, out = await post("stage", {"id": 7, "items": [sec], "yield_every": 1})
            assert out == {"staged": "7", "items": 1}
            st, out = await post("apply", {"staged": 7})
            assert out["applied"] == 1 and out["t1_ns"] >= out["t0_ns"] and "7" not in srv.staged
            # a second apply updates in place, keeping metadata the server owns
            uid = srv.state.get(R.SECRETS, NS, "m0")["metadata"]["uid"]
            sec2 = make_secret("m0", NS, version=2)
            sec2["metadata"]["labels"] = {"wave": "2"}
            st, out = await post("apply", {"items": [sec2, make_configmap("c0", NS)], "yield_every": 1})
            cur = srv.state.get(R.SECRETS, NS, "m0")
            assert out["applied"] == 2 and cur["metadata"]["uid"] == uid and cur["metadata"]["labels"] == {"wave": "2"}
            st, out = await post("markers/wait", {"want": [{"plural": "secrets", "value": sec2["data"]["version"],
                                                            "count": 1}], "timeout": 5, "times": True, "keyed": True})
            assert out["ok"] and list(out["counts"].values()) == [1] and "times" in out
            # seeding: a dependent owned by an existing template resolves the template's live UID
            t = srv.state.create(R.TEMPLATES, NS, make_template(3, NS))
            dep = make_secret("owned", NS)
            dep["__owner_template__"] = t["metadata"]["name"]
            st, out = await post("objects", {"items": [dep, make_secret("m0", NS)]})
            assert out["created"] == 1  # m0 exists already: skipped
            refs = srv.state.get(R.SECRETS, NS, "owned")["metadata"]["ownerReferences"]
            assert refs[0]["uid"] == t["metadata"]["uid"]
            st, out = await post("admission", {"prune_defaults": False, "sets": {}})
            assert st == 200
            st, out = await post("faults", {"compact": True})
            assert st == 200
            async with s.get(f"{url}/_fake/stats") as r:
                stats = await r.json()
            assert stats["name"] == "ctl" and stats["objects"]["core/secrets"] == 2
            async with s.post(f"{url}/_fake/nope", json={}) as r:
                assert r.status == 404
    finally:
        await srv.stop()


async def test_serve_entrypoint_exits_when_parent_is_gone(tmp_path):
    """`python -m ncc.fakeapi` as spawned by tests and benches, run in-process: markers, an admission field
    set, the port file, and the exit once the parent PID disappears."""
    import argparse
    import gc
    import subprocess
    import sys

    from ncc.fakeapi.server import serve
    dead = subprocess.Popen([sys.executable, "-c", "pass"])
    dead.wait()
    pf = tmp_path / "url"
    args = argparse.Namespace(name="served", token=None, bookmark_interval=5.0, crd_dir=None, host="127.0.0.1",
                              port=0, port_file=str(pf), tls_cert=None, tls_key=None, tls_client_ca=None,
                              prune_defaults=False, admission_set=['secrets=metadata.labels.hook="on"'],
                              parent_pid=dead.pid, marker=["secrets=data.version"])
    thresholds = gc.get_threshold()
    try:
        await asyncio.wait_for(serve(args), timeout=15)
    finally:
        gc.set_threshold(*thresholds)
        gc.unfreeze()
    assert pf.read_text().startswith("http://127.0.0.1:")


async def test_request_admission_seats_queue_inflight_and_service_time():
    """The APF / max-in-flight model (ncc/fakeapi/flowcontrol.py): requests beyond the seats wait in a bounded
    FIFO queue, a full queue, an expired wait or too many mutating requests are answered 429 with
    `Retry-After: 1`, and a write holds its seat for the service time."""
    import json as _json
    import time as _time

    import aiohttp

    srv = FakeApiServer(name="apf")
    url = await srv.start()
    path = f"{url}/api/v1/namespaces/{NS}/secrets"

    async def burst(session, n, tag):
        async def one(i):
            async with session.post(path, data=_json.dumps(make_secret(f"{tag}{i}", NS)),
                                    headers={"Content-Type": "application/json"}) as r:
                await r.read()
                return r.status, r.headers.get("Retry-After")
        return await asyncio.gather(*(one(i) for i in range(n)))

    try:
        async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0)) as session:
            srv.faults.update({"apf_seats": 2, "apf_queue": 2, "service_ms": 100})
            t0 = _time.monotonic()
            res = await burst(session, 10, "a")
            took = _time.monotonic() - t0
            assert sorted(s for s, _ in res) == [201] * 4 + [429] * 6
            assert all(ra == "1" for s, ra in res if s == 429)
            assert 0.19 <= took < 1.5  # two seats, four writes of 100 ms each: two rounds
            st = srv.flow.stats()
            assert st["admitted"] == 4 and st["queued"] == 2 and st["rejected_queue_full"] == 6
            assert st["max_executing"] == 2 and st["executing"] == 0 and st["waiting"] == 0
            assert sum(b[1] for b in st["by_second"]) == 10 and sum(b[2] for b in st["by_second"]) == 6
            # an expired wait for a seat is a 429 too
            srv.faults.update({"apf_seats": 1, "apf_queue": 5, "apf_queue_wait_s": 0.05, "service_ms": 200})
            res = await burst(session, 3, "b")
            assert sorted(s for s, _ in res) == [201, 429, 429]
            assert srv.flow.stats()["rejected_queue_wait"] == 2 and srv.flow.executing == 0
            # max-mutating-inflight without APF
            srv.faults.update({"apf_seats": 0, "max_mutating_inflight": 1, "service_ms": 100})
            res = await burst(session, 3, "c")
            assert sorted(s for s, _ in res) == [201, 429, 429]
            assert srv.flow.stats()["rejected_inflight"] == 2 and srv.flow.mutating == 0
            # reads are not mutating: not limited by max_mutating_inflight
            async with session.get(path) as r:
                assert r.status == 200
            srv.faults.update({"max_mutating_inflight": 0, "service_ms": 0})
            async with session.get(f"{url}/_fake/stats") as r:
                stats = await r.json()
            assert stats["flow"]["admitted"] >= 6 and stats["connections"]["api_max"] >= 1
            assert stats["requests"]["throttled"] == 10
    finally:
        await srv.stop()
