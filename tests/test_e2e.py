"""End-to-end: `App` against fake apiservers over real HTTP (Test_ControllerMain analogue, controller_test.go:1287-1336)."""
import asyncio
import logging

import pytest

from ncc.api import constants as C
from ncc.api import resources as R
from ncc.app import App
from ncc.kube import errors as E
from ncc.testing.env import FakeEnvironment
from ncc.testing.workload import make_configmap, make_secret, make_template, make_workgroup

NS = "nexus"


async def wait_for(pred, timeout=5.0, interval=0.02):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    last = None
    while loop.time() < end:
        try:
            last = await pred()
            if last:
                return last
        except E.NotFound:
            pass
        await asyncio.sleep(interval)
    raise AssertionError(f"condition not met within {timeout}s (last={last!r})")


async def mutate(client, rt, name, fn, attempts=20):
    """GET-modify-PUT with optimistic-concurrency retries (the controller writes status concurrently)."""
    for _ in range(attempts):
        cur = await client.get(rt, NS, name)
        fn(cur)
        try:
            return await client.update(rt, NS, cur)
        except E.Conflict:
            await asyncio.sleep(0.01)
    raise AssertionError(f"could not update {name}")


async def _get(client, rt, name):
    return await client.get(rt, NS, name)


class Running:
    def __init__(self, env, mode, **cfg_kw):
        self.app = App(env.app_config(mode=mode, **cfg_kw))
        self.stop = asyncio.Event()

    async def __aenter__(self):
        await self.app.build()
        self.task = asyncio.ensure_future(self.app.run(self.stop))
        await asyncio.wait_for(self.app.controller.ready.wait(), 10)
        return self.app

    async def __aexit__(self, *exc):
        self.stop.set()
        await asyncio.wait_for(self.task, 15)


@pytest.mark.parametrize("mode", ["compat", "native"])
async def test_controller_main_propagates_create_and_update(tmp_path, mode):
    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    try:
        t = make_template(0, NS)
        await cc.create(R.TEMPLATES, NS, t)
        async with Running(env, mode):
            # the reference's integration test allows 1 s for each propagation step
            await wait_for(lambda: _get(sc, R.TEMPLATES, "algo-00000"), timeout=1.0)
            await mutate(cc, R.TEMPLATES, "algo-00000", lambda o: o["spec"]["container"].__setitem__("versionTag",
                                                                                                  "v2.3.4"))

            async def propagated():
                o = await sc.get(R.TEMPLATES, NS, "algo-00000")
                return o["spec"]["container"]["versionTag"] == "v2.3.4"
            await wait_for(propagated, timeout=1.0)
            shard_t = await sc.get(R.TEMPLATES, NS, "algo-00000")
            assert shard_t["metadata"]["labels"] == C.owner_labels("controller-cluster")

            async def ready():
                o = await cc.get(R.TEMPLATES, NS, "algo-00000")
                conds = (o.get("status") or {}).get("conditions") or []
                return conds and conds[0]["status"] == "True" and o["status"]["syncedToClusters"] == ["shard-0"]
            await wait_for(ready, timeout=2.0)
    finally:
        await cc.close()
        await sc.close()
        await env.stop()


@pytest.mark.parametrize("mode,transport,ssa", [("compat", "fast", False), ("native", "fast", False),
                                                ("native", "aiohttp", False), ("native", "fast", True)])
async def test_dependents_fan_out_and_delete(tmp_path, mode, transport, ssa):
    env = await FakeEnvironment(2, str(tmp_path)).start()
    cc = env.controller_client()
    scs = [env.shard_client(i) for i in range(2)]
    try:
        await cc.create(R.SECRETS, NS, make_secret("s0", NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap("c0", NS))
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=["s0"], configmaps=["c0"]))
        await cc.create(R.WORKGROUPS, NS, make_workgroup("mi355x", NS))
        async with Running(env, mode, transport=transport, server_side_apply=ssa):
            for sc in scs:
                st = await wait_for(lambda sc=sc: _get(sc, R.TEMPLATES, "algo-00000"), timeout=3)
                sec = await wait_for(lambda sc=sc: _get(sc, R.SECRETS, "s0"), timeout=3)
                cm = await wait_for(lambda sc=sc: _get(sc, R.CONFIGMAPS, "c0"), timeout=3)
                await wait_for(lambda sc=sc: _get(sc, R.WORKGROUPS, "mi355x"), timeout=3)
                for dep in (sec, cm):
                    refs = dep["metadata"]["ownerReferences"]
                    assert [r["uid"] for r in refs] == [st["metadata"]["uid"]]
                    assert dep["metadata"]["labels"][C.LABEL_CONFIGURATION_OWNER] == "controller-cluster"
            ctrl_secret = await cc.get(R.SECRETS, NS, "s0")
            assert ctrl_secret["metadata"]["ownerReferences"][0]["kind"] == C.TEMPLATE_KIND

            # data change in the controller cluster propagates to every shard
            await mutate(cc, R.SECRETS, "s0", lambda o: o.__setitem__("data", {"token": "bmV3"}))
            for sc in scs:
                async def updated(sc=sc):
                    return (await sc.get(R.SECRETS, NS, "s0")).get("data") == {"token": "bmV3"}
                await wait_for(updated, timeout=3)

            # template deletion removes it from shards; shard GC collects the dependents
            await cc.delete(R.TEMPLATES, NS, "algo-00000")
            for sc in scs:
                async def gone(sc=sc):
                    try:
                        await sc.get(R.TEMPLATES, NS, "algo-00000")
                        return False
                    except E.NotFound:
                        pass
                    try:
                        await sc.get(R.SECRETS, NS, "s0")
                        return False
                    except E.NotFound:
                        return True
                await wait_for(gone, timeout=3)
    finally:
        await cc.close()
        for sc in scs:
            await sc.close()
        await env.stop()


async def test_native_repairs_shard_drift_and_workgroup_delete(tmp_path):
    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    try:
        await cc.create(R.TEMPLATES, NS, make_template(0, NS))
        await cc.create(R.WORKGROUPS, NS, make_workgroup("mi355x", NS))
        async with Running(env, "native"):
            st = await wait_for(lambda: _get(sc, R.TEMPLATES, "algo-00000"), timeout=2)
            # someone edits the shard copy: native mode watches shards and repairs it without waiting for resync
            await mutate(sc, R.TEMPLATES, "algo-00000", lambda o: o["spec"]["container"].__setitem__(
                "versionTag", "tampered"))

            async def repaired():
                o = await sc.get(R.TEMPLATES, NS, "algo-00000")
                return o["spec"]["container"]["versionTag"] == "v1.0.0"
            await wait_for(repaired, timeout=2)
            await wait_for(lambda: _get(sc, R.WORKGROUPS, "mi355x"), timeout=2)
            await cc.delete(R.WORKGROUPS, NS, "mi355x")

            async def wg_gone():
                try:
                    await sc.get(R.WORKGROUPS, NS, "mi355x")
                    return False
                except E.NotFound:
                    return True
            await wait_for(wg_gone, timeout=2)
    finally:
        await cc.close()
        await sc.close()
        await env.stop()


async def test_leader_election_failover(tmp_path):
    """Two replicas with `leader-elect`: only the Lease holder reconciles; the standby takes over when the
    leader shuts down (released Lease → immediate) and keeps propagating."""
    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    kw = dict(leader_elect=True, lease_duration=1.0, renew_deadline=0.6, retry_period=0.1)
    apps = [App(env.app_config(mode="native", **kw)) for _ in range(2)]
    stops = [asyncio.Event(), asyncio.Event()]
    try:
        await apps[0].build()
        t0 = asyncio.ensure_future(apps[0].run(stops[0]))
        await asyncio.wait_for(apps[0].controller.ready.wait(), 10)
        await apps[1].build()
        t1 = asyncio.ensure_future(apps[1].run(stops[1]))
        await asyncio.sleep(0.5)
        assert apps[0].elector.leading and not apps[1].elector.leading
        assert not apps[1].controller.ready.is_set() and apps[1]._ready()
        await cc.create(R.TEMPLATES, NS, make_template(0, NS))
        await wait_for(lambda: _get(sc, R.TEMPLATES, "algo-00000"), timeout=3)

        stops[0].set()
        await asyncio.wait_for(t0, 15)
        await asyncio.wait_for(apps[1].controller.ready.wait(), 10)
        assert apps[1].elector.leading
        lease = await cc.get(R.LEASES, NS, "nexus-configuration-controller")
        assert lease["spec"]["holderIdentity"] == apps[1].elector.identity
        await cc.create(R.TEMPLATES, NS, make_template(1, NS))
        await wait_for(lambda: _get(sc, R.TEMPLATES, "algo-00001"), timeout=3)
        stops[1].set()
        await asyncio.wait_for(t1, 15)
    finally:
        for s in stops:
            s.set()
        await cc.close()
        await sc.close()
        await env.stop()


async def test_warm_standby_takes_over_within_lease_duration(tmp_path):
    """A standby lists/watches every cluster and pre-spawns its executors (workers gated) before it holds
    the Lease.  When the leader dies without releasing the Lease, the first shard write of a new template
    version lands within lease-duration + 1 s, with 1k templates in the caches."""
    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    lease = 2.0
    kw = dict(leader_elect=True, lease_duration=lease, renew_deadline=1.2, retry_period=0.2)
    for i in range(1000):
        env.controller_server.state.create(R.TEMPLATES, NS, make_template(i, NS))
    apps = [App(env.app_config(mode="native", **kw)) for _ in range(2)]
    stops = [asyncio.Event(), asyncio.Event()]
    try:
        await apps[0].build()
        t0 = asyncio.ensure_future(apps[0].run(stops[0]))
        await asyncio.wait_for(apps[0].controller.ready.wait(), 10)
        await wait_for(lambda: asyncio.sleep(0, env.shard_servers[0].state.count(R.TEMPLATES) == 1000),
                       timeout=30)
        await apps[1].build()
        t1 = asyncio.ensure_future(apps[1].run(stops[1]))
        # the standby is warm: its caches and its executors' caches synced while it does not lead
        await asyncio.wait_for(apps[1].controller.caches_synced.wait(), 10)
        await wait_for(lambda: asyncio.sleep(0, apps[1].pool is not None and apps[1].pool.all_synced()), timeout=20)
        assert not apps[1].elector.leading and not apps[1].controller.ready.is_set()

        async def no_release():
            return False
        apps[0].elector.release = no_release  # the leader dies: its Lease is left to expire
        stops[0].set()
        await asyncio.wait_for(t0, 15)
        loop = asyncio.get_running_loop()
        t_dead = loop.time()
        await mutate(cc, R.TEMPLATES, "algo-00007", lambda o: o["spec"]["container"].__setitem__("versionTag", "v-new"))

        async def propagated():
            st = await sc.get(R.TEMPLATES, NS, "algo-00007")
            return st["spec"]["container"]["versionTag"] == "v-new"
        await wait_for(propagated, timeout=lease + 5, interval=0.01)
        took = loop.time() - t_dead
        assert apps[1].elector.leading and apps[1].standby_was_warm
        assert took < lease + 1.0, f"takeover to first shard write took {took:.2f}s"
        stops[1].set()
        await asyncio.wait_for(t1, 15)
    finally:
        for s in stops:
            s.set()
        await cc.close()
        await sc.close()
        await env.stop()


async def test_partitioned_executors_per_shard(tmp_path):
    """`executors-per-shard: 2`: two key-partitioned executors serve each shard; every template is synced
    exactly by its partition's owner and the coordinator still reports Ready for all."""
    from ncc.controller.executor import key_part
    env = await FakeEnvironment(2, str(tmp_path)).start()
    cc = env.controller_client()
    scs = [env.shard_client(i) for i in range(2)]
    try:
        T = 12
        for i in range(T):
            await cc.create(R.SECRETS, NS, make_secret(f"s{i}", NS))
            await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=[f"s{i}"], configmaps=[]))
        parts = {key_part(f"template/{NS}/algo-{i:05d}", 2) for i in range(T)}
        assert parts == {0, 1}  # the workload really exercises both partitions
        async with Running(env, "native", executors_per_shard=2) as app:
            assert len(app.pool.handles) == 4

            async def all_ready():
                items = (await cc.list(R.TEMPLATES, NS))["items"]
                return len(items) == T and all(
                    (o.get("status") or {}).get("syncedToClusters") == ["shard-0", "shard-1"] and
                    o["status"]["conditions"][0]["status"] == "True" for o in items)
            await wait_for(all_ready, timeout=10)
            for sc in scs:
                assert len((await sc.list(R.TEMPLATES, NS))["items"]) == T
                assert len((await sc.list(R.SECRETS, NS))["items"]) == T
    finally:
        await cc.close()
        for sc in scs:
            await sc.close()
        await env.stop()


@pytest.mark.parametrize("executors", [0, -1])
async def test_native_converges_under_faults(tmp_path, executors):
    """Failure detection/recovery soak: with 30 % of shard writes failing (5xx), injected latency, and
    every shard watch dropped mid-run, the native controller still converges every template on every
    shard (per-key backoff retries, watch resume/relist), and statuses end Ready once faults clear."""
    env = await FakeEnvironment(2, str(tmp_path)).start()
    cc = env.controller_client()
    scs = [env.shard_client(i) for i in range(2)]
    T = 20
    try:
        async with aiohttp_session() as s:
            for srv in env.shard_servers:
                async with s.post(srv.url + "/_fake/faults", json={"error_rate": 0.3, "error_code": 503,
                                                                   "latency_ms": 2, "jitter_ms": 3}) as r:
                    await r.json()
            async with Running(env, "native", executors=executors, failure_rate_max_delay=0.2):
                for i in range(T):
                    await cc.create(R.SECRETS, NS, make_secret(f"s{i}", NS))
                    await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=[f"s{i}"], configmaps=[]))
                await asyncio.sleep(0.3)
                for srv in env.shard_servers:  # cut every watch stream; informers resume from their last RV
                    async with s.post(srv.url + "/_fake/faults", json={"drop_watches": True}) as r:
                        await r.json()

                async def shards_converged():
                    for sc in scs:
                        if len((await sc.list(R.TEMPLATES, NS))["items"]) != T:
                            return False
                        if len((await sc.list(R.SECRETS, NS))["items"]) != T:
                            return False
                    return True
                await wait_for(shards_converged, timeout=20, interval=0.1)
                for srv in env.shard_servers:
                    async with s.post(srv.url + "/_fake/faults", json={"error_rate": 0.0, "latency_ms": 0,
                                                                       "jitter_ms": 0}) as r:
                        await r.json()

                async def all_ready():
                    items = (await cc.list(R.TEMPLATES, NS))["items"]
                    return len(items) == T and all(
                        o.get("status", {}).get("conditions", [{}])[0].get("status") == "True" and
                        o["status"]["syncedToClusters"] == ["shard-0", "shard-1"] for o in items)
                await wait_for(all_ready, timeout=20, interval=0.1)
    finally:
        await cc.close()
        for sc in scs:
            await sc.close()
        await env.stop()


def aiohttp_session():
    import aiohttp
    return aiohttp.ClientSession()


async def test_partitioned_executors_shared_dependents(tmp_path):
    """Templates in different key partitions sharing one Secret/ConfigMap: each partition's executor adds
    its own ownerRef (refetch on AlreadyExists/Conflict), and a data change reaches the shard once."""
    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    try:
        T = 12
        await cc.create(R.SECRETS, NS, make_secret("shared", NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap("shared-cm", NS))
        for i in range(T):
            await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=["shared"], configmaps=["shared-cm"]))
        async with Running(env, "native", executors_per_shard=2):
            async def owned_by_all():
                uids = {o["metadata"]["uid"] for o in (await sc.list(R.TEMPLATES, NS))["items"]}
                if len(uids) != T:
                    return False
                for rt, nm in ((R.SECRETS, "shared"), (R.CONFIGMAPS, "shared-cm")):
                    o = await sc.get(rt, NS, nm)
                    if {r["uid"] for r in o["metadata"].get("ownerReferences") or ()} != uids:
                        return False
                return True
            await wait_for(owned_by_all, timeout=15, interval=0.05)
            await mutate(cc, R.SECRETS, "shared", lambda o: o.__setitem__("data", {"token": "c2hhcmVk"}))

            async def updated():
                return (await sc.get(R.SECRETS, NS, "shared")).get("data") == {"token": "c2hhcmVk"}
            await wait_for(updated, timeout=10)

            async def all_ready():
                items = (await cc.list(R.TEMPLATES, NS))["items"]
                return all((o.get("status") or {}).get("conditions", [{}])[0].get("status") == "True"
                           for o in items)
            await wait_for(all_ready, timeout=10)
    finally:
        await cc.close()
        await sc.close()
        await env.stop()


@pytest.mark.parametrize("executors", [0, -1])
async def test_shard_hot_reload(tmp_path, executors):
    """Adding/removing a `<cluster>.kubeconfig` in the shards directory takes effect without a restart
    (the reference loads shards once at startup, main.go:73)."""
    import os
    import shutil
    env = await FakeEnvironment(2, str(tmp_path)).start()
    cc, s0, s1 = env.controller_client(), env.shard_client(0), env.shard_client(1)
    parked = os.path.join(str(tmp_path), "shard-1.kubeconfig.parked")
    shutil.move(os.path.join(env.shard_dir, "shard-1.kubeconfig"), parked)

    async def status_is(shards):
        o = await cc.get(R.TEMPLATES, NS, "algo-00000")
        st = o.get("status") or {}
        return st.get("syncedToClusters") == shards and st["conditions"][0]["status"] == "True"
    try:
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=[], configmaps=[]))
        async with Running(env, "native", executors=executors, shard_reload_period=0) as app:
            await wait_for(lambda: status_is(["shard-0"]), timeout=5)
            shutil.move(parked, os.path.join(env.shard_dir, "shard-1.kubeconfig"))
            diff = await app.reload_shards()
            assert diff == {"added": ["shard-1"], "removed": [], "changed": []}
            await wait_for(lambda: _get(s1, R.TEMPLATES, "algo-00000"), timeout=10)
            await wait_for(lambda: status_is(["shard-0", "shard-1"]), timeout=10)
            os.remove(os.path.join(env.shard_dir, "shard-0.kubeconfig"))
            assert (await app.reload_shards())["removed"] == ["shard-0"]
            await wait_for(lambda: status_is(["shard-1"]), timeout=10)
            assert await app.reload_shards() == {}
    finally:
        for c in (cc, s0, s1):
            await c.close()
        await env.stop()


async def test_partition_filter_keeps_newly_referenced_dependent(tmp_path):
    """Executors drop controller-side Secrets owned only by other partitions' templates before decoding.
    A template of the *other* partition that starts referencing such a Secret must still sync it (the
    reverse index keeps it, and a filtered-out reference is fetched once), and later data changes must
    reach the shard through both partitions."""
    from ncc.controller.executor import key_part
    from ncc.controller.executor import partition_owner_filter
    keep = partition_owner_filter(0, 2, referenced=lambda ns, name: name == "wanted")
    names = [f"algo-{i:05d}" for i in range(40)]
    mine = next(n for n in names if key_part(f"template/{NS}/{n}", 2) == 0)
    other = next(n for n in names if key_part(f"template/{NS}/{n}", 2) == 1)
    assert keep(NS, "x", ()) and keep(NS, "x", (mine,)) and keep(NS, "wanted", (other,))
    assert not keep(NS, "x", (other,))

    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    try:
        ia, ib = int(mine.split("-")[1]), int(other.split("-")[1])
        await cc.create(R.SECRETS, NS, make_secret("s-shared", NS))
        await cc.create(R.TEMPLATES, NS, make_template(ia, NS, secrets=["s-shared"]))
        async with Running(env, "native", executors_per_shard=2):
            async def owned(uids):
                o = await sc.get(R.SECRETS, NS, "s-shared")
                return {r["uid"] for r in o["metadata"].get("ownerReferences") or ()} == uids
            await wait_for(lambda: _get(sc, R.TEMPLATES, mine), timeout=5)
            ua = (await sc.get(R.TEMPLATES, NS, mine))["metadata"]["uid"]
            await wait_for(lambda: owned({ua}), timeout=5)
            # now a template of the other partition references the Secret owned only by the first one
            await cc.create(R.TEMPLATES, NS, make_template(ib, NS, secrets=["s-shared"]))
            await wait_for(lambda: _get(sc, R.TEMPLATES, other), timeout=5)
            ub = (await sc.get(R.TEMPLATES, NS, other))["metadata"]["uid"]
            await wait_for(lambda: owned({ua, ub}), timeout=5)
            await mutate(cc, R.SECRETS, "s-shared", lambda o: o.__setitem__("data", {"token": "bmV3LXZhbA=="}))

            async def updated():
                return (await sc.get(R.SECRETS, NS, "s-shared")).get("data") == {"token": "bmV3LXZhbA=="}
            await wait_for(updated, timeout=5)

            async def both_ready():
                for n in (mine, other):
                    st = (await cc.get(R.TEMPLATES, NS, n)).get("status") or {}
                    if (st.get("conditions") or [{}])[0].get("status") != "True":
                        return False
                return True
            await wait_for(both_ready, timeout=5)
    finally:
        await cc.close()
        await sc.close()
        await env.stop()


@pytest.mark.parametrize("impl", ["native", "python"])
async def test_partitioned_coordinators(tmp_path, impl, monkeypatch):
    """coordinator-partitions=2: the template keys are split between the parent coordinator and one child
    coordinator process; the parent's executors serve both, and the reports on the child's keys are
    forwarded to it.  Every template still becomes Ready, shared dependents are adopted by all their
    templates, and a killed child is restarted, resynced and resumes its keys."""
    import os
    import signal
    from ncc.controller.executor import key_part
    env = await FakeEnvironment(2, str(tmp_path)).start()
    cc = env.controller_client()
    scs = [env.shard_client(i) for i in range(2)]
    T = 12
    try:
        await cc.create(R.SECRETS, NS, make_secret("shared", NS))
        for i in range(T):
            await cc.create(R.CONFIGMAPS, NS, make_configmap(f"c{i}", NS))
            await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=["shared"], configmaps=[f"c{i}"]))
        parts = {key_part(f"template/{NS}/algo-{i:05d}", 2) for i in range(T)}
        assert parts == {0, 1}, "the workload must exercise both coordinator partitions"
        monkeypatch.delenv("NCC_EXECUTOR_IMPL", raising=False)
        async with Running(env, "native", coordinator_partitions=2, executors_per_shard=2,
                           executor_impl=impl) as app:
            assert app.coord_part == (0, 2) and app.partitions is not None and app.executor_impl == impl
            assert len(app.pool.handles) == 2 * 2 and app.topology()["executor_processes"] == 4

            async def all_ready(tag=None):
                items = (await cc.list(R.TEMPLATES, NS))["items"]
                if len(items) != T:
                    return False
                for o in items:
                    st = o.get("status") or {}
                    if (st.get("conditions") or [{}])[0].get("status") != "True" or \
                            st.get("syncedToClusters") != ["shard-0", "shard-1"]:
                        return False
                    if tag and o["spec"]["container"]["versionTag"] != tag:
                        return False
                return True
            await wait_for(all_ready, timeout=20, interval=0.05)
            await wait_for(lambda: asyncio.sleep(0, app._ready()), timeout=10)
            owners = {r["name"] for r in (await cc.get(R.SECRETS, NS, "shared"))["metadata"]["ownerReferences"]}
            assert owners == {f"algo-{i:05d}" for i in range(T)}
            for sc in scs:
                uids = {o["metadata"]["uid"] for o in (await sc.list(R.TEMPLATES, NS))["items"]}
                sec = await sc.get(R.SECRETS, NS, "shared")
                assert {r["uid"] for r in sec["metadata"]["ownerReferences"]} == uids and len(uids) == T
            # Events go out asynchronously after the status write (the broadcaster's writers, as client-go's
            # sink goroutine): a template can be Ready before its Synced Event is posted — wait for them
            want = {f"algo-{i:05d}" for i in range(T)}
            synced = set()

            async def all_synced_events():
                nonlocal synced
                events = (await cc.list(R.EVENTS, NS))["items"]
                synced = {e["involvedObject"]["name"] for e in events if e["reason"] == C.SUCCESS_SYNCED}
                return synced == want
            try:
                await wait_for(all_synced_events, timeout=10, interval=0.05)
            except AssertionError:
                raise AssertionError(f"Synced Events missing for {sorted(want - synced)}") from None
            assert app.partitions.forwarded > 0  # the child's statuses came from forwarded reports

            # kill the child coordinator: it is restarted and keeps serving its partition
            child = app.partitions.handles[0]
            old_pid = child.proc.pid
            os.kill(old_pid, signal.SIGKILL)
            await wait_for(lambda: asyncio.sleep(0, child.proc is not None and child.proc.pid != old_pid
                                                 and child.ready.is_set()), timeout=20, interval=0.05)
            for i in range(T):
                await mutate(cc, R.TEMPLATES, f"algo-{i:05d}",
                             lambda o: o["spec"]["container"].__setitem__("versionTag", "v-part"))

            async def propagated():
                for sc in scs:
                    for o in (await sc.list(R.TEMPLATES, NS))["items"]:
                        if o["spec"]["container"]["versionTag"] != "v-part":
                            return False
                return True
            await wait_for(propagated, timeout=20, interval=0.05)
            await wait_for(lambda: all_ready("v-part"), timeout=20, interval=0.05)
    finally:
        await cc.close()
        for sc in scs:
            await sc.close()
        await env.stop()


def test_partitioned_coordinators_share_the_executors(tmp_path, monkeypatch):
    """C coordinators share one set of executors (the parent's: k per shard, every key) instead of each
    running its own: a shard apiserver serves k executors' watches whatever C is."""
    import asyncio as aio
    from ncc.app import App
    monkeypatch.delenv("NCC_COORDINATOR_PART", raising=False)

    async def go():
        env = await FakeEnvironment(4, str(tmp_path)).start()
        try:
            app = App(env.app_config(mode="native", coordinator_partitions=2, executors_per_shard=4))
            await app.build()
            assert app.coord_part == (0, 2) and app.per_shard == 4 and app.n_executors == 4
            await app.factory.stop()
        finally:
            await env.stop()
    aio.run(go())


@pytest.mark.parametrize("impl", ["native", "python"])
async def test_watch_relay_one_list_and_watch_per_kind_and_relist(tmp_path, impl, monkeypatch):
    """Native mode with 2 shards × 2 executors: the controller apiserver serves one LIST and one WATCH per
    kind (the coordinator's; executors are fed by its watch relay).  After a 410 relist of the coordinator
    (watch history compacted while the apiserver was unreachable), executors get a fresh snapshot: a
    template changed and one deleted during the gap both reach the shards, with no executor LIST."""
    monkeypatch.delenv("NCC_EXECUTOR_IMPL", raising=False)
    env = await FakeEnvironment(2, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(1)
    st = env.controller_server.state
    for i in range(20):
        st.create(R.SECRETS, NS, make_secret(f"s{i}", NS))
        st.create(R.CONFIGMAPS, NS, make_configmap(f"c{i}", NS))
        st.create(R.TEMPLATES, NS, make_template(i, NS, secrets=[f"s{i}"], configmaps=[f"c{i}"]))
    try:
        async with Running(env, "native", executors_per_shard=2, executor_impl=impl) as app:
            assert app.relay is not None and len(app.pool.handles) == 4 and app.executor_impl == impl

            async def all_synced():
                return all(s.state.count(R.TEMPLATES) == 20 and s.state.count(R.SECRETS) == 20
                           for s in env.shard_servers)
            await wait_for(all_synced, timeout=20)
            await wait_for(lambda: asyncio.sleep(0, st.stats["watch"] >= 4), timeout=5)
            await asyncio.sleep(0.2)
            assert st.stats["list"] == 4 and st.stats["watch"] == 4, st.stats

            srv = env.controller_server
            srv.faults.update({"down": True})
            srv.drop_watches()
            cur = st.get(R.TEMPLATES, NS, "algo-00003")
            upd = dict(cur, spec=dict(cur["spec"], container=dict(cur["spec"]["container"], versionTag="v-gap")))
            st.update(R.TEMPLATES, NS, upd)
            st.delete(R.TEMPLATES, NS, "algo-00004")
            st.compact()
            srv.faults.update({"down": False})

            async def caught_up():
                t = await sc.get(R.TEMPLATES, NS, "algo-00003")
                if t["spec"]["container"]["versionTag"] != "v-gap":
                    return False
                try:
                    await sc.get(R.TEMPLATES, NS, "algo-00004")
                    return False
                except E.NotFound:
                    return True
            await wait_for(caught_up, timeout=20)
            assert st.stats["list"] == 8, st.stats  # one relist per kind, by the coordinator only
            assert app.relay.stats["snapshots"] >= 8
    finally:
        await cc.close()
        await sc.close()
        await env.stop()


async def test_reload_with_changed_kubeconfig_reaches_native_executor(tmp_path, monkeypatch):
    """a shard whose kubeconfig changes (a rotated CA, a moved server) gets a C++ executor
    configured from the *new* file — the coordinator's credential cache must not hand it the old one."""
    import os
    import shutil
    from ncc.controller.native_executor import binary_path
    if binary_path() is None:
        pytest.skip("ncc/bin/ncc-executor is not built")
    monkeypatch.delenv("NCC_EXECUTOR_IMPL", raising=False)
    env = await FakeEnvironment(2, str(tmp_path)).start()
    cc = env.controller_client()
    parked = os.path.join(str(tmp_path), "shard-1.kubeconfig.parked")
    shutil.move(os.path.join(env.shard_dir, "shard-1.kubeconfig"), parked)
    try:
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=[], configmaps=[]))
        async with Running(env, "native", executor_impl="native", shard_reload_period=0) as app:
            assert app.executor_impl == "native"
            await wait_for(lambda: asyncio.sleep(0, env.shard_servers[0].state.count(R.TEMPLATES) == 1), timeout=10)
            assert env.shard_servers[1].state.count(R.TEMPLATES) == 0
            with open(os.path.join(env.shard_dir, "shard-0.kubeconfig"), "w") as f:
                f.write(env.kubeconfig(env.shard_urls[1], "shard-0"))  # "shard-0" now lives on server 1
            assert await app.reload_shards() == {"added": [], "removed": [], "changed": ["shard-0"]}
            await wait_for(lambda: asyncio.sleep(0, env.shard_servers[1].state.count(R.TEMPLATES) == 1), timeout=15)
            assert app.native_cfg.creds["shard-0"].cfg.server == env.shard_urls[1]
    finally:
        await cc.close()
        await env.stop()


async def test_python_executor_fallback_is_loud(tmp_path, monkeypatch, caplog):
    """under `executor-impl: auto`, a coordinator that cannot run the C++ executors (here:
    the watch relay switched off) runs the Python ones with a Warning, the executor_native gauge at 0, and the
    reason in /readyz?verbose and /debug/state — not silently.  With the relay on, the gauge is 1."""
    import aiohttp

    from ncc.controller.native_executor import binary_path
    if binary_path() is None:
        pytest.skip("the C++ executor is not built")
    monkeypatch.delenv("NCC_EXECUTOR_IMPL", raising=False)

    class Gauges:
        def __init__(self):
            self.g = {}

        def gauge(self, name, value, tags=None):
            self.g[name] = value

        def __getattr__(self, _name):
            return lambda *a, **k: None

    env = await FakeEnvironment(1, str(tmp_path)).start()
    try:
        for relay, impl in ((False, "python"), (True, "native")):
            caplog.clear()
            metrics = Gauges()
            app = App(env.app_config(mode="native", watch_relay=relay, health_bind_address="127.0.0.1:0"),
                      metrics=metrics)
            stop = asyncio.Event()
            with caplog.at_level(logging.WARNING, logger="ncc"):
                await app.build()
                task = asyncio.ensure_future(app.run(stop))
                try:
                    await asyncio.wait_for(app.controller.ready.wait(), 15)
                    assert app.executor_impl == impl
                    assert metrics.g[C.EXECUTOR_NATIVE_METRIC] == (1 if impl == "native" else 0)
                    async with aiohttp.ClientSession() as s:
                        async with s.get(f"http://127.0.0.1:{app.ops.port}/readyz?verbose") as r:
                            text = await r.text()
                    assert r.status == 200 and "[+]shard-executors " + impl in text and "readyz check passed" in text
                    fallback = [m for m in caplog.messages if "Python implementation runs instead" in m]
                    if impl == "python":
                        assert "the watch relay is off" in text and fallback
                        assert app.debug_state()["executor_fallback"] == "the watch relay is off"
                    else:
                        assert "fallback" not in text and not fallback
                finally:
                    stop.set()
                    await asyncio.wait_for(task, 20)
    finally:
        await env.stop()


async def test_managed_fields_are_not_cached_and_survive_updates(tmp_path, monkeypatch):
    """metadata.managedFields (server-side apply's field ownership; hundreds of bytes per object on a real
    apiserver) is dropped from the C++ executor's cached shard objects and the coordinator's metadata-only store:
    an update that omits it leaves the server's as it is (kube-apiserver semantics, mirrored by the fake), so a
    shard copy with managedFields and stale data is brought up to date and keeps them."""
    from ncc.controller.native_executor import binary_path
    if binary_path() is None:
        pytest.skip("the C++ executor is not built")
    monkeypatch.delenv("NCC_EXECUTOR_IMPL", raising=False)
    mf = [{"manager": "kubectl", "operation": "Update", "apiVersion": "v1", "time": "2025-01-01T00:00:00Z",
           "fieldsType": "FieldsV1", "fieldsV1": {"f:data": {".": {}, "f:version": {}}}}]
    env = await FakeEnvironment(1, str(tmp_path)).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    try:
        s = make_secret("s0", NS, version=2)
        s["metadata"]["managedFields"] = mf
        await cc.create(R.SECRETS, NS, s)
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=["s0"], configmaps=[]))
        async with Running(env, "native", executor_impl="native") as app:
            assert app.executor_impl == "native"

            async def synced():
                try:
                    o = await sc.get(R.SECRETS, NS, "s0")
                except E.NotFound:
                    return False
                return o["data"] == s["data"]
            await wait_for(synced, timeout=5.0)
            # the stale-data update path: the shard copy gains managedFields of its own, then the source changes
            o = await sc.get(R.SECRETS, NS, "s0")
            o["metadata"]["managedFields"] = mf
            await sc.update(R.SECRETS, NS, o)
            await mutate(cc, R.SECRETS, "s0", lambda x: x.__setitem__("data", {"version": "Mw=="}))

            async def updated():
                return (await sc.get(R.SECRETS, NS, "s0"))["data"] == {"version": "Mw=="}
            await wait_for(updated, timeout=5.0)
            assert (await sc.get(R.SECRETS, NS, "s0"))["metadata"].get("managedFields") == mf
            cached = app.controller.secret_informer.store.get(NS, "s0")
            assert cached is not None and "managedFields" not in cached["metadata"]
    finally:
        await env.stop()
