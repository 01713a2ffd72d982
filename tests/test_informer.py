"""SharedInformer behaviour: list/watch, relist on 410 with tombstones, resync, transforms, mutation overlay."""
import asyncio

from ncc.api import resources as R
from ncc.cache.informer import DeletedFinalStateUnknown, Informer
from ncc.cache.store import Store
from ncc.fakeapi.server import FakeApiServer
from ncc.fakeapi.storage import ClusterState
from ncc.kube.kubeconfig import ClusterConfig
from ncc.kube.rest import RestClient
from ncc.testing.fake_client import FakeClient
from ncc.testing.workload import make_secret

NS = "nexus"


class Rec:
    def __init__(self):
        self.log = []

    def add(self, o):
        self.log.append(("add", o["metadata"]["name"]))

    def update(self, old, new):
        self.log.append(("update", new["metadata"]["name"], old is new))

    def delete(self, o):
        if isinstance(o, DeletedFinalStateUnknown):
            self.log.append(("tombstone", o.key.name))
        else:
            self.log.append(("delete", o["metadata"]["name"]))


async def wait_until(pred, timeout=3.0):
    end = asyncio.get_running_loop().time() + timeout
    while asyncio.get_running_loop().time() < end:
        if pred():
            return True
        await asyncio.sleep(0.01)
    raise AssertionError("timeout")


async def test_list_then_watch_events_in_order():
    state = ClusterState()
    state.create(R.SECRETS, NS, make_secret("pre", NS))
    client = FakeClient(state, simple=False)
    inf = Informer(client, R.SECRETS, NS)
    rec = Rec()
    inf.add_event_handler(rec.add, rec.update, rec.delete)
    inf.start()
    assert await inf.wait_for_sync(2)
    state.create(R.SECRETS, NS, make_secret("a", NS))
    cur = state.get(R.SECRETS, NS, "a")
    state.update(R.SECRETS, NS, dict(cur, data={"k": "dg=="}))
    state.delete(R.SECRETS, NS, "pre")
    await wait_until(lambda: len(rec.log) == 4)
    assert rec.log == [("add", "pre"), ("add", "a"), ("update", "a", False), ("delete", "pre")]
    assert inf.lister.get(NS, "a")["data"] == {"k": "dg=="}
    await inf.stop()


async def test_relist_after_gone_emits_tombstones():
    state = ClusterState(history=2)
    for n in ("a", "b"):
        state.create(R.SECRETS, NS, make_secret(n, NS))
    srv = FakeApiServer(state=state)
    url = await srv.start()
    client = RestClient(ClusterConfig(server=url))
    inf = Informer(client, R.SECRETS, NS)
    rec = Rec()
    inf.add_event_handler(rec.add, rec.update, rec.delete)
    inf.start()
    assert await inf.wait_for_sync(2)
    # while the watch is down, history is compacted and "a" disappears: the resume gets 410 → relist
    srv.drop_watches()
    state.compact()
    state.delete(R.SECRETS, NS, "a")
    state.compact()
    state.create(R.SECRETS, NS, make_secret("c", NS))
    state.compact()
    await wait_until(lambda: ("tombstone", "a") in rec.log and ("add", "c") in rec.log)
    assert inf.relists >= 2
    assert sorted(o["metadata"]["name"] for o in inf.lister.list()) == ["b", "c"]
    await inf.stop()
    await client.close()
    await srv.stop()


async def test_resync_redelivers_same_object():
    state = ClusterState()
    state.create(R.SECRETS, NS, make_secret("a", NS))
    inf = Informer(FakeClient(state, simple=False), R.SECRETS, NS, resync_period=0.05)
    rec = Rec()
    inf.add_event_handler(rec.add, rec.update, rec.delete)
    inf.start()
    await wait_until(lambda: ("update", "a", True) in rec.log)
    await inf.stop()


async def test_transform_and_async_handler():
    state = ClusterState()
    state.create(R.SECRETS, NS, make_secret("a", NS))
    inf = Informer(FakeClient(state, simple=False), R.SECRETS, NS,
                   transform=lambda o: {"metadata": o["metadata"], "slim": True})
    seen = []

    async def on_add(o):
        await asyncio.sleep(0)
        seen.append(o)
    inf.add_event_handler(on_add=on_add)
    inf.start()
    await wait_until(lambda: seen)
    assert seen[0]["slim"] is True and "data" not in inf.lister.get(NS, "a")
    await inf.stop()


async def test_informer_recovers_from_transport_errors():
    srv = FakeApiServer()
    url = await srv.start()
    client = RestClient(ClusterConfig(server=url))
    inf = Informer(client, R.SECRETS, NS)
    srv.faults.update({"down": True, "write_only": False})
    inf.start()
    await asyncio.sleep(0.3)
    assert not inf.has_synced() and inf.last_error is not None
    srv.faults.update({"down": False})
    assert await inf.wait_for_sync(5)
    await inf.stop()
    await client.close()
    await srv.stop()


async def test_answering_ends_an_outage_backoff_once():
    """After an outage the list/watch backoff grows towards 30 s.  When the owner's other requests are
    answered again (`Informer.answering`, set by ncc/shards/shard.py), the sleeping informer retries at once
    — only once per outage, so an endpoint that keeps failing still backs off."""
    srv = FakeApiServer()
    url = await srv.start()
    client = RestClient(ClusterConfig(server=url))
    inf = Informer(client, R.SECRETS, NS)
    inf.answering = asyncio.Event()
    srv.faults.update({"down": True, "write_only": False})
    inf.start()
    await asyncio.sleep(2.0)  # failures at 0, ~0.8, ~2.4 s: the next wait is ~3.2 s
    assert not inf.has_synced()
    srv.faults.update({"down": False})
    t0 = asyncio.get_running_loop().time()
    inf.answering.set()  # e.g. a shard write succeeded
    assert await inf.wait_for_sync(1.0)
    assert asyncio.get_running_loop().time() - t0 < 1.0
    await inf.stop()
    await client.close()
    await srv.stop()


def test_store_indices_and_mutation_overlay():
    s = Store()
    s.add_indexer("owner", lambda o: [r["uid"] for r in o["metadata"].get("ownerReferences", [])])
    o = make_secret("a", NS)
    o["metadata"].update(resourceVersion="5", ownerReferences=[{"uid": "u1"}])
    s.upsert(o)
    assert [x["metadata"]["name"] for x in s.by_index("owner", "u1")] == ["a"]
    newer = dict(o, metadata=dict(o["metadata"], resourceVersion="7", ownerReferences=[]))
    s.assume(newer)
    assert s.get(NS, "a")["metadata"]["resourceVersion"] == "7"     # overlay visible before the watch catches up
    s.assume(dict(o, metadata=dict(o["metadata"], resourceVersion="6")))  # older than overlay: ignored
    assert s.get(NS, "a")["metadata"]["resourceVersion"] == "7"
    s.upsert(dict(newer))                                            # informer catches up → overlay dropped
    assert s.get(NS, "a")["metadata"]["resourceVersion"] == "7" and not s._assumed
    assert s.by_index("owner", "u1") == []
    added, updated, deleted = s.replace([make_secret("b", NS)])
    assert [x["metadata"]["name"] for x in added] == ["b"] and [x["metadata"]["name"] for x in deleted] == ["a"]


async def test_key_filter_drops_foreign_keys_on_list_and_watch():
    """Partitioned executors: a key filter keeps other partitions' objects out of the store — off the wire
    (native scanner, raw watch over HTTP) and on the decoded path (in-memory client)."""
    for http in (True, False):
        state = ClusterState()
        state.create(R.SECRETS, NS, make_secret("keep-0", NS))
        state.create(R.SECRETS, NS, make_secret("drop-0", NS))
        srv = None
        if http:
            srv = FakeApiServer(state=state)
            client = RestClient(ClusterConfig(server=await srv.start()))
        else:
            client = FakeClient(state, simple=False)
        inf = Informer(client, R.SECRETS, NS, key_filter=lambda ns, name: ns == NS and name.startswith("keep"))
        rec = Rec()
        inf.add_event_handler(rec.add, rec.update, rec.delete)
        inf.start()
        assert await inf.wait_for_sync(2)
        for n in ("drop-1", "keep-1"):
            state.create(R.SECRETS, NS, make_secret(n, NS))
        state.delete(R.SECRETS, NS, "drop-0")
        state.delete(R.SECRETS, NS, "keep-0")
        await wait_until(lambda: len(rec.log) == 3)
        assert rec.log == [("add", "keep-0"), ("add", "keep-1"), ("delete", "keep-0")]
        assert [o["metadata"]["name"] for o in inf.lister.list()] == ["keep-1"]
        await wait_until(lambda: inf.last_rv == str(state.rv))  # filtered events still advance the RV
        assert inf.filtered >= 2
        await inf.stop()
        if srv is not None:
            await client.close()
            await srv.stop()


async def test_owner_filter_and_parked_echoes():
    """Owner filter (partitioned executors) and in-flight write tracking: a watch event that overtakes
    the response of our own write is parked undecoded and settled by `end_write`."""
    from ncc.api.objects import ObjectKey
    state = ClusterState()
    srv = FakeApiServer(state=state)
    client = RestClient(ClusterConfig(server=await srv.start()))

    def owned(name, owners):
        s = make_secret(name, NS)
        s["metadata"]["ownerReferences"] = [{"apiVersion": "v1", "kind": "NexusAlgorithmTemplate", "name": o,
                                             "uid": f"u-{o}"} for o in owners]
        return s
    try:
        state.create(R.SECRETS, NS, owned("a", ["mine"]))
        state.create(R.SECRETS, NS, owned("b", ["other"]))
        state.create(R.SECRETS, NS, owned("c", []))
        inf = Informer(client, R.SECRETS, NS, owner_filter=lambda ns, name, owners: not owners or "mine" in owners)
        rec = Rec()
        inf.add_event_handler(rec.add, rec.update, rec.delete)
        inf.start()
        assert await inf.wait_for_sync(2)
        assert sorted(o["metadata"]["name"] for o in inf.lister.list()) == ["a", "c"]
        state.create(R.SECRETS, NS, owned("d", ["other", "mine"]))
        cur = state.get(R.SECRETS, NS, "a")
        state.update(R.SECRETS, NS, dict(cur, metadata=dict(cur["metadata"], ownerReferences=owned(
            "a", ["other"])["metadata"]["ownerReferences"])))
        await wait_until(lambda: inf.lister.try_get(NS, "d") is not None and inf.lister.try_get(NS, "a") is None)
        assert rec.log[-1] == ("add", "d")  # "a" left the partition silently

        # our write's echo overtakes its response: parked, then confirmed without dispatch
        key = ObjectKey(NS, "c")
        inf.begin_write(key)
        cur = state.get(R.SECRETS, NS, "c")
        res = state.update(R.SECRETS, NS, dict(cur, data={"k": "MQ=="}))
        await wait_until(lambda: key in inf._stash)
        n_log, echoes = len(rec.log), inf.echoes
        await inf.end_write(key, res)
        assert inf.echoes == echoes + 1 and len(rec.log) == n_log
        assert inf.lister.get(NS, "c")["data"] == {"k": "MQ=="}

        # a newer foreign write parked behind our (older) response is applied when the write ends
        inf.begin_write(key)
        cur = state.get(R.SECRETS, NS, "c")
        ours = state.update(R.SECRETS, NS, dict(cur, data={"k": "Mg=="}))
        theirs = state.update(R.SECRETS, NS, dict(ours, data={"k": "Mw=="}))
        await wait_until(lambda: key in inf._stash and inf._stash[key][0] == theirs["metadata"]["resourceVersion"])
        await inf.end_write(key, ours)
        assert inf.lister.get(NS, "c")["data"] == {"k": "Mw=="}
        assert rec.log[-1] == ("update", "c", False)
        await inf.stop()
    finally:
        await client.close()
        await srv.stop()


async def test_metadata_only_skips_payload_updates_but_not_owner_changes():
    state = ClusterState()
    srv = FakeApiServer(state=state)
    client = RestClient(ClusterConfig(server=await srv.start()))
    try:
        state.create(R.SECRETS, NS, make_secret("s", NS))
        inf = Informer(client, R.SECRETS, NS, transform=lambda o: {k: v for k, v in o.items() if k != "data"})
        inf.metadata_only = True
        rec = Rec()
        inf.add_event_handler(rec.add, rec.update, rec.delete)
        inf.start()
        assert await inf.wait_for_sync(2)
        cur = state.get(R.SECRETS, NS, "s")
        cur = state.update(R.SECRETS, NS, dict(cur, data={"k": "MQ=="}))  # payload only → skipped
        ref = {"apiVersion": "v1", "kind": "NexusAlgorithmTemplate", "name": "t", "uid": "u1"}
        cur = state.update(R.SECRETS, NS, dict(cur, metadata=dict(cur["metadata"], ownerReferences=[ref])))
        cur = state.update(R.SECRETS, NS, dict(cur, metadata=dict(cur["metadata"], ownerReferences=[
            dict(ref, uid="u2")])))  # same owner name, new uid (template re-created) → delivered
        await wait_until(lambda: inf.last_rv == str(state.rv))
        assert rec.log == [("add", "s"), ("update", "s", False), ("update", "s", False)]
        assert inf.lister.get(NS, "s")["metadata"]["ownerReferences"][0]["uid"] == "u2"
        assert "data" not in inf.lister.get(NS, "s") and inf.filtered == 1
        await inf.stop()
    finally:
        await client.close()
        await srv.stop()


def test_store_index_tracks_value_changes_and_relists():
    from ncc.cache.store import Store
    from ncc.testing.workload import make_template
    st = Store()
    st.add_indexer("secret", lambda t: [f"nexus/{n}" for n in
                                        [e.get("secretRef", {}).get("name") for e in
                                         t["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"]] if n])
    t = make_template(0, "nexus", secrets=["a"])
    st.upsert(t)
    assert [o["metadata"]["name"] for o in st.by_index("secret", "nexus/a")] == ["algo-00000"]
    t2 = make_template(0, "nexus", secrets=["a"], version="v9")  # same references: buckets untouched
    st.upsert(t2)
    assert st.by_index("secret", "nexus/a")[0]["spec"]["container"]["versionTag"] == "v9"
    st.upsert(make_template(0, "nexus", secrets=["b"]))  # moved to another bucket
    assert st.by_index("secret", "nexus/a") == [] and len(st.by_index("secret", "nexus/b")) == 1
    st.upsert(make_template(0, "nexus", secrets=[]))  # no references left
    assert st.by_index("secret", "nexus/b") == [] and st._index_vals["secret"] == {}
    st.replace([make_template(1, "nexus", secrets=["c"])])
    assert len(st.by_index("secret", "nexus/c")) == 1
    st.delete(make_template(1, "nexus", secrets=["c"]))
    assert st.by_index("secret", "nexus/c") == [] and st._index_vals["secret"] == {}


async def test_list_resource_version_semantics():
    """Reflector semantics: cold-start LIST at resourceVersion "0" (watch cache), continuation pages carry
    only the token, and after 410 Gone the relist is a consistent read ("")."""
    import asyncio as aio
    from ncc.cache.informer import Informer
    from ncc.kube import errors as E2

    calls = []

    class Client:
        cluster_name = "c"
        watches = 0

        async def list(self, rt, ns, *, label_selector=None, limit=None, continue_token=None,
                       resource_version=None):
            calls.append((resource_version, continue_token))
            if continue_token is None and len(calls) == 1:
                return {"items": [], "metadata": {"resourceVersion": "5", "continue": "page2"}}
            return {"items": [], "metadata": {"resourceVersion": "5"}}

        async def watch(self, rt, ns, **kw):
            Client.watches += 1
            if Client.watches == 1:
                raise E2.Gone("expired")
            await aio.sleep(3600)
            yield  # pragma: no cover

    inf = Informer(Client(), R.SECRETS, "nexus")
    task = aio.ensure_future(inf._run())
    for _ in range(200):
        if len(calls) >= 3:
            break
        await aio.sleep(0.01)
    task.cancel()
    await aio.gather(task, return_exceptions=True)
    assert calls[:3] == [("0", None), (None, "page2"), ("", None)]
