"""Native-mode behaviours that deliberately differ from the reference."""
import msgpack
import pytest

from ncc.api import constants as C
from ncc.api import resources as R
from ncc.cache.informer import Informer
from ncc.controller.controller import Controller, make_key
from ncc.controller.events import FakeRecorder
from ncc.controller.options import ControllerOptions
from ncc.controller.reconcile import ShardSyncError, slim_data, slim_spec
from ncc.fakeapi.storage import ClusterState
from ncc.kube import errors as E
from ncc.shards.shard import Shard
from ncc.testing.fake_client import FakeClient
from ncc.testing.workload import make_configmap, make_secret, make_template, make_workgroup

NS = "nexus"
ALIAS = "ctl"


class Env:
    """Controller + N shards on in-memory clusters with real apiserver semantics (UIDs, RVs, GC)."""

    def __init__(self, n_shards=2, **opt):
        self.cstate = ClusterState("controller")
        self.cclient = FakeClient(self.cstate, cluster_name="controller", simple=False)
        self.sstates = [ClusterState(f"s{i}") for i in range(n_shards)]
        self.sclients = [FakeClient(s, cluster_name=f"s{i}", simple=False) for i, s in enumerate(self.sstates)]
        self.opts = ControllerOptions.native(native_queue=False, coalesce_window=0.0, **opt)

    def build(self, role="all"):
        self.opts.role = role
        infs = {rt: Informer(self.cclient, rt, NS) for rt in (R.TEMPLATES, R.WORKGROUPS, R.SECRETS, R.CONFIGMAPS)}
        slim = {R.TEMPLATES: slim_spec, R.WORKGROUPS: slim_spec, R.SECRETS: slim_data, R.CONFIGMAPS: slim_data}
        self.shards = [Shard(ALIAS, f"s{i}", c, NS, assume_writes=True, sync_binary_data=True, transforms=slim)
                       for i, c in enumerate(self.sclients)]
        self.recorder = FakeRecorder()
        self.ctl = Controller(alias=ALIAS, namespace=NS, client=self.cclient,
                              shards=self.shards if role != "coordinator" else [],
                              template_informer=infs[R.TEMPLATES], workgroup_informer=infs[R.WORKGROUPS],
                              secret_informer=infs[R.SECRETS], configmap_informer=infs[R.CONFIGMAPS],
                              options=self.opts, recorder=self.recorder,
                              shard_names=[f"s{i}" for i in range(len(self.sstates))])
        self.refresh()
        return self.ctl

    def refresh(self):
        """Simulate informers catching up: replace every store with the cluster's current content."""
        for rt, inf in ((R.TEMPLATES, self.ctl.template_informer), (R.WORKGROUPS, self.ctl.workgroup_informer),
                        (R.SECRETS, self.ctl.secret_informer), (R.CONFIGMAPS, self.ctl.configmap_informer)):
            inf.store.replace(self.cstate.list(rt, NS)["items"])
            inf._synced.set()
        for sh, st in zip(self.shards, self.sstates):
            for rt, inf in ((R.TEMPLATES, sh.template_informer), (R.WORKGROUPS, sh.workgroup_informer),
                            (R.SECRETS, sh.secret_informer), (R.CONFIGMAPS, sh.configmap_informer)):
                inf.store.replace(st.list(rt, NS)["items"])
                inf._synced.set()

    def seed(self, i=0, secrets=("s",), configmaps=("c",)):
        for s in secrets:
            self.cstate.create(R.SECRETS, NS, make_secret(s, NS))
        for c in configmaps:
            self.cstate.create(R.CONFIGMAPS, NS, make_configmap(c, NS))
        return self.cstate.create(R.TEMPLATES, NS, make_template(i, NS, secrets=list(secrets),
                                                                 configmaps=list(configmaps)))


async def test_fanout_to_all_shards_and_status():
    env = Env(3)
    t = env.seed()
    ctl = env.build()
    await ctl.sync_template(NS, t["metadata"]["name"])
    for st in env.sstates:
        assert st.count(R.TEMPLATES) == 1 and st.count(R.SECRETS) == 1 and st.count(R.CONFIGMAPS) == 1
        sec = st.get(R.SECRETS, NS, "s")
        assert sec["metadata"]["ownerReferences"][0]["uid"] == st.get(R.TEMPLATES, NS, t["metadata"]["name"])[
            "metadata"]["uid"]
    got = env.cstate.get(R.TEMPLATES, NS, t["metadata"]["name"])
    assert got["status"]["conditions"][0]["status"] == "True"
    assert got["status"]["syncedToClusters"] == ["s0", "s1", "s2"]
    assert env.recorder.events[-1].startswith("Normal Synced")
    # second pass is a no-op: no writes, no event (event_on_noop=False)
    n_actions = [len(c.writes()) for c in env.sclients]
    env.refresh()
    env.recorder.events.clear()
    await ctl.sync_template(NS, t["metadata"]["name"])
    assert [len(c.writes()) for c in env.sclients] == n_actions and env.recorder.events == []


async def test_single_put_for_data_and_owner():
    env = Env(1)
    t = env.seed()
    ctl = env.build()
    # shard already has the secret, owned by some other template, with stale data
    other = env.sstates[0].create(R.TEMPLATES, NS, make_template(99, NS))
    sec = make_secret("s", NS, version=42)
    sec["metadata"]["ownerReferences"] = [{"apiVersion": C.API_VERSION, "kind": C.TEMPLATE_KIND,
                                           "name": other["metadata"]["name"], "uid": other["metadata"]["uid"]}]
    env.sstates[0].create(R.SECRETS, NS, sec)
    env.refresh()
    await ctl.sync_template(NS, t["metadata"]["name"])
    secret_writes = [a for a in env.sclients[0].writes() if a.resource.plural == "secrets"]
    assert len(secret_writes) == 1 and secret_writes[0].verb == "update"
    live = env.sstates[0].get(R.SECRETS, NS, "s")
    assert live["data"] == env.cstate.get(R.SECRETS, NS, "s")["data"]
    assert len(live["metadata"]["ownerReferences"]) == 2


async def test_failure_isolation_reports_failed_shard():
    env = Env(2)
    t = env.seed()
    ctl = env.build()
    env.sclients[1].prepend_reactor("create", "*", lambda a: (True, None, E.ServiceUnavailable("shard down")))
    with pytest.raises(ShardSyncError) as ei:
        await ctl.sync_template(NS, t["metadata"]["name"])
    assert set(ei.value.failures) == {"s1"}
    assert env.sstates[0].count(R.TEMPLATES) == 1 and env.sstates[1].count(R.TEMPLATES) == 0
    st = env.cstate.get(R.TEMPLATES, NS, t["metadata"]["name"])["status"]
    assert st["conditions"][0]["status"] == "False" and "s1" in st["conditions"][0]["message"]
    assert st["syncedToClusters"] == ["s0"]
    env.sclients[1].reactors.clear()
    env.refresh()
    await ctl.sync_template(NS, t["metadata"]["name"])
    st = env.cstate.get(R.TEMPLATES, NS, t["metadata"]["name"])["status"]
    assert st["conditions"][0]["status"] == "True" and st["syncedToClusters"] == ["s0", "s1"]


async def test_write_race_already_exists_is_tolerated():
    env = Env(1)
    t = env.seed()
    ctl = env.build()
    # the shard template exists but our cache has not seen it yet
    env.sstates[0].create(R.TEMPLATES, NS, dict(make_template(0, NS), metadata={
        "name": t["metadata"]["name"], "namespace": NS, "labels": C.owner_labels(ALIAS)}))
    await ctl.sync_template(NS, t["metadata"]["name"])
    assert env.sstates[0].count(R.SECRETS) == 1


async def test_queued_delete_retries_and_orphan_sweep():
    env = Env(2)
    t = env.seed()
    ctl = env.build()
    name = t["metadata"]["name"]
    await ctl.sync_template(NS, name)
    env.cstate.delete(R.TEMPLATES, NS, name)
    env.refresh()
    ctl._handle_template_delete(t)
    assert len(ctl.queue) == 1
    env.sclients[1].prepend_reactor("delete", "*", lambda a: (True, None, E.InternalError("boom")))
    with pytest.raises(E.InternalError):
        await ctl.sync_template(NS, name)
    assert env.sstates[0].count(R.TEMPLATES) == 0 and env.sstates[1].count(R.TEMPLATES) == 1
    env.sclients[1].reactors.clear()
    env.refresh()
    await ctl.sync_template(NS, name)          # retry succeeds; dependents are garbage-collected
    assert env.sstates[1].count(R.TEMPLATES) == 0 and env.sstates[1].count(R.SECRETS) == 0
    # orphan sweep: labelled shard objects without a controller object are removed; foreign ones are kept
    mine = make_template(5, NS)
    mine["metadata"]["labels"] = C.owner_labels(ALIAS)
    env.sstates[0].create(R.TEMPLATES, NS, mine)
    env.sstates[0].create(R.TEMPLATES, NS, make_template(6, NS))
    env.refresh()
    while len(ctl.queue):
        ctl.queue.try_get()
    assert ctl.sweep_orphans() == 1
    await ctl.sync_template(NS, mine["metadata"]["name"])
    names = [o["metadata"]["name"] for o in env.sstates[0].list(R.TEMPLATES, NS)["items"]]
    assert names == ["algo-00006"]


async def test_binary_data_and_workgroup_delete_propagation():
    env = Env(1)
    cm = make_configmap("c", NS)
    cm["binaryData"] = {"blob": "AAEC"}
    env.cstate.create(R.CONFIGMAPS, NS, cm)
    t = env.cstate.create(R.TEMPLATES, NS, make_template(0, NS, configmaps=["c"]))
    w = env.cstate.create(R.WORKGROUPS, NS, make_workgroup("mi355x", NS))
    ctl = env.build()
    await ctl.sync_template(NS, t["metadata"]["name"])
    await ctl.sync_workgroup(NS, "mi355x")
    assert env.sstates[0].get(R.CONFIGMAPS, NS, "c")["binaryData"] == {"blob": "AAEC"}
    assert env.sstates[0].count(R.WORKGROUPS) == 1
    env.cstate.delete(R.WORKGROUPS, NS, "mi355x")
    env.refresh()
    ctl._on_workgroup_delete(w)
    await ctl.sync_workgroup(NS, "mi355x")
    assert env.sstates[0].count(R.WORKGROUPS) == 0


async def test_executor_refuses_missing_references_and_reports():
    env = Env(2)
    t = env.cstate.create(R.TEMPLATES, NS, make_template(0, NS, secrets=["missing"]))
    ctl = env.build(role="executor")
    reports = []
    ctl.reporter = reports.append
    with pytest.raises(E.NotFound):
        await ctl.sync_template(NS, t["metadata"]["name"])
    assert all(st.count(R.TEMPLATES) == 0 for st in env.sstates) and reports == []
    env.cstate.create(R.SECRETS, NS, make_secret("missing", NS))
    env.refresh()
    await ctl.sync_template(NS, t["metadata"]["name"])
    assert reports and reports[-1]["r"] == {"s0": None, "s1": None}
    assert reports[-1]["k"] == make_key(C.KIND_TEMPLATE, NS, t["metadata"]["name"])
    # executors never write to the controller cluster
    assert env.cclient.writes() == []


async def test_coordinator_waits_for_all_shard_reports():
    env = Env(2)
    t = env.seed()
    ctl = env.build(role="coordinator")
    name = t["metadata"]["name"]
    key = make_key(C.KIND_TEMPLATE, NS, name)
    await ctl.sync_template(NS, name)
    st = env.cstate.get(R.TEMPLATES, NS, name)["status"]
    assert st["conditions"][0]["status"] == "False"          # initialized, waiting for executors
    env.refresh()
    cur = env.cstate.get(R.TEMPLATES, NS, name)["metadata"]
    ctl.on_executor_message(0, {"t": "report", "k": key, "u": cur["uid"], "g": cur["generation"],
                                "r": {"s0": None}, "w": True})
    await ctl.sync_template(NS, name)
    assert env.cstate.get(R.TEMPLATES, NS, name)["status"]["conditions"][0]["status"] == "False"
    ctl.on_executor_message(1, {"t": "report", "k": key, "u": cur["uid"], "g": cur["generation"],
                                "r": {"s1": "ServiceUnavailable: down"}, "w": False})
    env.refresh()
    await ctl.sync_template(NS, name)
    st = env.cstate.get(R.TEMPLATES, NS, name)["status"]
    assert st["conditions"][0]["status"] == "False" and "s1" in st["conditions"][0]["message"]
    ctl.on_executor_message(1, {"t": "report", "k": key, "u": cur["uid"], "g": cur["generation"],
                                "r": {"s1": None}, "w": True})
    env.refresh()
    await ctl.sync_template(NS, name)
    st = env.cstate.get(R.TEMPLATES, NS, name)["status"]
    assert st["conditions"][0]["status"] == "True" and st["syncedToClusters"] == ["s0", "s1"]
    assert any(e.startswith("Normal Synced") for e in env.recorder.events)
    # a report about an older incarnation (different UID) does not count
    assert ctl.shard_readiness(key, {"metadata": {"uid": "other", "generation": 1}}) is None


async def test_server_side_apply_writes():
    """`server_side_apply`: every shard write is one apply PATCH (no GET/PUT, no resourceVersion);
    other owners' refs survive, drift is corrected, a rogue (unowned) object still blocks."""
    env = Env(1, server_side_apply=True)
    t = env.seed()
    name = t["metadata"]["name"]
    ctl = env.build()
    other = env.sstates[0].create(R.TEMPLATES, NS, make_template(99, NS))
    sec = make_secret("s", NS, version=42)
    sec["metadata"]["ownerReferences"] = [{"apiVersion": C.API_VERSION, "kind": C.TEMPLATE_KIND,
                                           "name": other["metadata"]["name"], "uid": other["metadata"]["uid"]}]
    env.sstates[0].create(R.SECRETS, NS, sec)
    env.refresh()
    await ctl.sync_template(NS, name)
    writes = env.sclients[0].writes()
    assert writes and all(a.verb == "patch" for a in writes)
    live = env.sstates[0].get(R.SECRETS, NS, "s")
    assert live["data"] == env.cstate.get(R.SECRETS, NS, "s")["data"]
    assert len(live["metadata"]["ownerReferences"]) == 2
    assert env.sstates[0].get(R.CONFIGMAPS, NS, "c")["metadata"]["labels"] == C.owner_labels(ALIAS)
    assert env.cstate.get(R.TEMPLATES, NS, name)["status"]["syncedToClusters"] == ["s0"]
    # spec drift on the shard is re-applied
    st = env.sstates[0].get(R.TEMPLATES, NS, name)
    st["spec"]["container"]["image"] = "drifted"
    env.sstates[0].update(R.TEMPLATES, NS, st)
    env.refresh()
    await ctl.sync_template(NS, name)
    assert env.sstates[0].get(R.TEMPLATES, NS, name)["spec"] == env.cstate.get(R.TEMPLATES, NS, name)["spec"]
    # a rogue configmap (no owner refs) is never overwritten
    env.cstate.create(R.CONFIGMAPS, NS, make_configmap("rogue", NS))
    env.sstates[0].create(R.CONFIGMAPS, NS, make_configmap("rogue", NS, version=7))
    t2 = env.cstate.create(R.TEMPLATES, NS, make_template(5, NS, secrets=[], configmaps=["rogue"]))
    env.refresh()
    with pytest.raises(Exception):
        await ctl.sync_template(NS, t2["metadata"]["name"])
    assert env.sstates[0].get(R.CONFIGMAPS, NS, "rogue")["data"] != env.cstate.get(R.CONFIGMAPS, NS, "rogue")["data"]


@pytest.mark.parametrize("concurrent", [False, True])
async def test_server_side_apply_refused_template_still_fails_the_pass(concurrent):
    """A refused shard-template apply (422) lets the new dependents go out — the shard template keeps its UID —
    but the pass fails with the apply's error, whichever way the dependents are written; the dependents come
    from the source template's references, since the shard template still has the old spec."""
    env = Env(1, server_side_apply=True, concurrent_dependents=concurrent)
    t = env.seed()
    name = t["metadata"]["name"]
    ctl = env.build()
    await ctl.sync_template(NS, name)
    env.cstate.create(R.SECRETS, NS, make_secret("s2", NS))
    src = env.cstate.get(R.TEMPLATES, NS, name)
    src["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"].append({"secretRef": {"name": "s2"}})
    env.cstate.update(R.TEMPLATES, NS, src)
    env.refresh()
    env.sclients[0].prepend_reactor("patch", "nexusalgorithmtemplates",
                                    lambda a: (True, None, E.Invalid("spec: refused")))
    with pytest.raises(ShardSyncError) as ei:
        await ctl.sync_template(NS, name)
    assert isinstance(ei.value.failures["s0"], E.Invalid)
    assert env.sstates[0].get(R.SECRETS, NS, "s2") is not None
    st = env.cstate.get(R.TEMPLATES, NS, name)["status"]
    assert st["conditions"][0]["status"] == "False" and st["syncedToClusters"] == []


async def test_response_light_writes_match_server_state():
    """Slim-cache shards publish their own request body (plus the RV/UID scanned from the response): the
    cached slim object must equal what slim-transforming the server's stored object would give."""
    from ncc.fakeapi.server import FakeApiServer
    from ncc.kube.kubeconfig import ClusterConfig
    from ncc.kube.rest import RestClient
    from ncc.api.fingerprint import SLIM_FP
    srv = FakeApiServer(name="s0")
    client = RestClient(ClusterConfig(server=await srv.start()), cluster_name="s0")
    slim = {R.TEMPLATES: slim_spec, R.WORKGROUPS: slim_spec, R.SECRETS: slim_data, R.CONFIGMAPS: slim_data}
    sh = Shard(ALIAS, "s0", client, NS, assume_writes=True, sync_binary_data=True, transforms=slim)
    try:
        assert sh._write_meta is not None
        t = make_template(1, NS)
        st = await sh.create_template(t["metadata"]["name"], NS, t["spec"], C.FIELD_MANAGER)
        live = srv.state.get(R.TEMPLATES, NS, t["metadata"]["name"])
        assert st["metadata"]["uid"] == live["metadata"]["uid"]
        assert st["metadata"]["resourceVersion"] == live["metadata"]["resourceVersion"]
        assert st[SLIM_FP] == slim_spec(live)[SLIM_FP] and "spec" not in st
        sec = await sh.create_secret(st, make_secret("s", NS), C.FIELD_MANAGER)
        cm = make_configmap("c", NS)
        cm["binaryData"] = {"b": "AAE="}
        cmo = await sh.create_configmap(st, cm, C.FIELD_MANAGER)
        sec2 = await sh.update_secret(sec, {"token": "bmV3"}, None, C.FIELD_MANAGER)
        for got, rt, nm in ((sec2, R.SECRETS, "s"), (cmo, R.CONFIGMAPS, "c")):
            live = srv.state.get(rt, NS, nm)
            want = slim_data(live)
            assert got[SLIM_FP] == want[SLIM_FP]
            assert got["metadata"]["resourceVersion"] == live["metadata"]["resourceVersion"]
            assert got["metadata"]["uid"] == live["metadata"]["uid"]
            assert got["metadata"]["ownerReferences"] == live["metadata"]["ownerReferences"]
            assert sh.secret_lister.try_get(NS, "s") is sec2 if rt is R.SECRETS else True
        assert srv.state.get(R.SECRETS, NS, "s")["data"] == {"token": "bmV3"}
    finally:
        await client.close()
        await srv.stop()


async def test_secret_type_change_recreates_shard_copy():
    env = Env(1)
    t = env.seed()
    ctl = env.build()
    name = t["metadata"]["name"]
    await ctl.sync_template(NS, name)
    old_uid = env.sstates[0].get(R.SECRETS, NS, "s")["metadata"]["uid"]
    src = env.cstate.get(R.SECRETS, NS, "s")
    env.cstate.update(R.SECRETS, NS, dict(src, type="kubernetes.io/dockerconfigjson"))
    env.refresh()
    await ctl.sync_template(NS, name)
    live = env.sstates[0].get(R.SECRETS, NS, "s")
    assert live["type"] == "kubernetes.io/dockerconfigjson" and live["metadata"]["uid"] != old_uid
    st_uid = env.sstates[0].get(R.TEMPLATES, NS, name)["metadata"]["uid"]
    assert [r["uid"] for r in live["metadata"]["ownerReferences"]] == [st_uid]


async def test_rogue_event_on_template_and_adoption_switch():
    env = Env(1, controller_adoption=False)
    t = env.seed()
    env.sstates[0].create(R.CONFIGMAPS, NS, make_configmap("c", NS, version=3))  # rogue: no ownerRefs
    ctl = env.build()
    with pytest.raises(ShardSyncError):
        await ctl.sync_template(NS, t["metadata"]["name"])
    ev = [e for e in env.recorder.events if "ErrResourceExists" in e]
    assert ev and "ConfigMap" in ev[0] and 'shard "s0"' in ev[0]
    # controller-side dependents were not adopted (no GC coupling to the template)
    assert not env.cstate.get(R.SECRETS, NS, "s")["metadata"].get("ownerReferences")
    assert not env.cstate.get(R.CONFIGMAPS, NS, "c")["metadata"].get("ownerReferences")


def test_write_target_resolves_the_written_object():
    from ncc.controller.reconcile import _write_target
    st = {"metadata": {"name": "algo-1", "namespace": "ns1"}}
    src = {"metadata": {"name": "sec", "namespace": "ctl"}}
    assert _write_target("create_secret", (st, src, "fm")) == ("ns1", "sec")
    assert _write_target("create_configmap", (st, src, "fm")) == ("ns1", "sec")
    assert _write_target("update_secret", (dict(src), None, None, "fm")) == ("ctl", "sec")
    assert _write_target("create_template", ("algo-1", "ns1", {}, "fm")) == ("ns1", "algo-1")
    assert _write_target("update_template", (st, {}, "fm")) == ("ns1", "algo-1")


async def test_operational_metrics():
    from ncc.telemetry.statsd import MemoryMetrics
    env = Env(1)
    t = env.seed()
    ctl = env.build()
    ctl.metrics = MemoryMetrics()
    env.sclients[0].prepend_reactor("create", "*", lambda a: (True, None, E.ServiceUnavailable("down")))
    ctl.queue.add(make_key(C.KIND_TEMPLATE, NS, t["metadata"]["name"]))
    assert await ctl.process_next_work_item()
    v = ctl.metrics.values
    assert v[C.RECONCILE_ERRORS_METRIC] == [1.0] and v[C.WORKQUEUE_LENGTH_METRIC] and v[C.RECONCILE_LATENCY_METRIC]
    # coordinator side: an executor report carrying a shard error is counted per shard
    ctl.on_executor_message(0, {"t": "report", "k": make_key(C.KIND_TEMPLATE, NS, "x"), "u": "u", "g": 1,
                                "r": {"s0": "ServiceUnavailable: down"}, "w": False})
    assert v[C.SHARD_SYNC_ERRORS_METRIC] == [1.0]


async def test_adoption_cache_rechecks_after_dependent_events():
    """adoption_cache: a second pass over the same template version skips the adoption check, but a
    dependent event (e.g. the Secret re-created without our ownerRef) invalidates it."""
    env = Env(1)
    t = env.seed()
    name, key = t["metadata"]["name"], make_key(C.KIND_TEMPLATE, NS, t["metadata"]["name"])
    ctl = env.build()
    await ctl.sync_template(NS, name)
    assert env.cstate.get(R.SECRETS, NS, "s")["metadata"]["ownerReferences"][0]["name"] == name
    env.refresh()
    cur = ctl.template_lister.get(NS, name)
    assert ctl._adopted[key] == cur["metadata"]["resourceVersion"]
    calls = []
    orig = ctl.adopt_references

    async def spy(tpl):
        calls.append(tpl["metadata"]["name"])
        return await orig(tpl)
    ctl.adopt_references = spy
    await ctl.sync_template(NS, name)
    assert calls == []  # unchanged template version, no dependent event: no re-check

    # the Secret is replaced by one without ownerRefs; its informer event invalidates the cache
    env.cstate.delete(R.SECRETS, NS, "s")
    fresh = env.cstate.create(R.SECRETS, NS, make_secret("s", NS))
    env.refresh()
    ctl._on_dependent(fresh, "secret")
    assert key not in ctl._adopted
    await ctl.sync_template(NS, name)
    assert calls == [name]
    assert env.cstate.get(R.SECRETS, NS, "s")["metadata"]["ownerReferences"][0]["name"] == name

    # a new template version with the same references inherits the adoption mark
    old = ctl.template_lister.get(NS, name)
    new = dict(old, metadata=dict(old["metadata"], resourceVersion="999999"))
    ctl._adopted[key] = old["metadata"]["resourceVersion"]
    ctl._on_crd_update(old, new, C.KIND_TEMPLATE)
    assert ctl._adopted[key] == "999999"
    changed = dict(new, metadata=dict(new["metadata"], resourceVersion="1000000"),
                   spec=dict(new["spec"], runtimeEnvironment={"mappedEnvironmentVariables": []}))
    ctl._on_crd_update(new, changed, C.KIND_TEMPLATE)
    assert ctl._adopted[key] == "999999"  # references changed: the new version is not marked


async def test_coordinator_template_handler_is_native_and_skips_the_early_pass():
    """The template informer's on_update in the coordinator is the native decision (`ReportTable.template_update`)
    when the extension is loaded: a resync is filtered, a spec update of an adopted template whose reports are
    not in is skipped, and one whose reports are in is enqueued."""
    env = Env(2)
    t = env.seed()
    ctl = env.build(role="coordinator")
    if not hasattr(ctl.reports, "template_update"):
        pytest.skip("native extension not built")
    name = t["metadata"]["name"]
    key = make_key(C.KIND_TEMPLATE, NS, name)
    await ctl.sync_template(NS, name)
    env.refresh()
    handler = ctl.template_informer._handlers[0].on_update
    assert handler.__qualname__.endswith("_template_update_handler.<locals>.on_update")
    old = ctl.template_lister.get(NS, name)
    handler(old, old)
    assert len(ctl.queue) == 0 and ctl.queue.core.waiting() == 0
    new = dict(old, metadata=dict(old["metadata"], resourceVersion="900", generation=old["metadata"]["generation"] + 1),
               spec=dict(old["spec"], container=dict(old["spec"]["container"], versionTag="v-next")))
    handler(old, new)
    assert ctl.stats["early_passes_skipped"] == 1 and ctl.queue.core.waiting() == 0 and len(ctl.queue) == 0
    assert ctl._adopted[key] == "900"  # same references: the new version stays adopted
    m = new["metadata"]
    for i in range(2):
        ctl.reports.feed(msgpack.packb({"t": "report", "k": key, "u": m["uid"], "g": m["generation"],
                                        "r": {f"s{i}": None}, "w": False}), False)
    newer = dict(new, metadata=dict(new["metadata"], resourceVersion="901"),
                 spec=dict(new["spec"], container=dict(new["spec"]["container"], versionTag="v-next2")))
    handler(new, newer)  # every shard has reported on this generation: a pass is due
    assert ctl.stats["early_passes_skipped"] == 1 and ctl.queue.core.waiting() + len(ctl.queue) == 1


async def test_coordinator_skips_early_pass_until_reports_complete():
    """A spec update of an initialised, adopted template is not reconciled by the coordinator on its
    informer event (nothing to do before the executors report); the last report enqueues it — and if
    every report is already in when the event arrives, the event enqueues it."""
    env = Env(2)
    t = env.seed()
    ctl = env.build(role="coordinator")
    name = t["metadata"]["name"]
    key = make_key(C.KIND_TEMPLATE, NS, name)
    await ctl.sync_template(NS, name)
    env.refresh()
    old = ctl.template_lister.get(NS, name)
    ctl._on_crd_update(old, old, C.KIND_TEMPLATE)  # resync: filtered
    assert len(ctl.queue) == 0 and ctl.queue.core.waiting() == 0
    new = dict(old, metadata=dict(old["metadata"], resourceVersion="900", generation=old["metadata"]["generation"] + 1),
               spec=dict(old["spec"], container=dict(old["spec"]["container"], versionTag="v-next")))
    ctl._on_crd_update(old, new, C.KIND_TEMPLATE)
    assert ctl.stats["early_passes_skipped"] == 1 and ctl.queue.core.waiting() == 0 and len(ctl.queue) == 0
    m = new["metadata"]
    for i in range(2):
        ctl.on_executor_message(i, {"t": "report", "k": key, "u": m["uid"], "g": m["generation"],
                                    "r": {f"s{i}": None}, "w": True})
    assert ctl._inline_keys == {key}  # the last report completed the set: finished in the next batch
    ctl._inline_timer.cancel()
    ctl._flush_inline()  # workers not started: no inline finish, a queued pass instead
    assert ctl.queue.core.waiting() + len(ctl.queue) == 1 and ctl.stats["inline_finishes"] == 0
    # reports already complete for the next version: the informer event itself enqueues
    ctl.queue.shutdown()
    ctl2 = env.build(role="coordinator")
    ctl2._adopted[key] = new["metadata"]["resourceVersion"]
    newer = dict(new, metadata=dict(m, resourceVersion="901", generation=m["generation"] + 1))
    for i in range(2):
        ctl2.on_executor_message(i, {"t": "report", "k": key, "u": m["uid"], "g": m["generation"] + 1,
                                     "r": {f"s{i}": None}, "w": True})
    before = ctl2.queue.core.waiting() + len(ctl2.queue)
    ctl2._on_crd_update(new, newer, C.KIND_TEMPLATE)
    assert ctl2.stats["early_passes_skipped"] == 0 and ctl2.queue.core.waiting() + len(ctl2.queue) >= before


async def test_coordinator_finishes_complete_reports_inline():
    """A complete report set for an initialised, adopted template whose status already says Ready only needs
    the Synced Event: it is recorded without a queued pass.  Anything else (a status change, a failed shard,
    a pass already queued) goes through the work queue."""
    env = Env(2)
    t = env.seed()
    ctl = env.build(role="coordinator")
    name = t["metadata"]["name"]
    key = make_key(C.KIND_TEMPLATE, NS, name)
    ctl.ready.set()  # workers "running"

    def report(gen, errs=(None, None), wrote=True):
        cur = ctl.template_lister.get(NS, name)["metadata"]
        for i in range(2):
            ctl.on_executor_message(i, {"t": "report", "k": key, "u": cur["uid"], "g": gen,
                                        "r": {f"s{i}": errs[i]}, "w": wrote})
        ctl._inline_timer.cancel()
        ctl._flush_inline()

    await ctl.sync_template(NS, name)  # initialising status + adoption; no reports yet
    env.refresh()
    gen = ctl.template_lister.get(NS, name)["metadata"]["generation"]
    report(gen)  # status still "initializing": a real pass must write Ready
    assert len(ctl.queue) == 1 and ctl.stats["inline_finishes"] == 0
    assert ctl.queue.try_get() == key
    await ctl.sync_template(NS, name)
    ctl.queue.done(key)
    env.refresh()
    cur = ctl.template_lister.get(NS, name)
    assert cur["status"]["conditions"][0]["status"] == C.CONDITION_TRUE
    # a new version: the adoption mark follows it, every shard reports success, the status stays Ready
    spec = dict(cur["spec"], container=dict(cur["spec"]["container"], versionTag="v-next"))
    new = env.cstate.update(R.TEMPLATES, NS, dict(cur, spec=spec))
    ctl._on_crd_update(cur, new, C.KIND_TEMPLATE)
    env.refresh()
    events = len(env.recorder.events)
    report(new["metadata"]["generation"])
    assert ctl.stats["inline_finishes"] == 1 and len(ctl.queue) == 0 and ctl.queue.core.waiting() == 0
    assert env.recorder.events[events:] == [f"{C.EVENT_TYPE_NORMAL} {C.SUCCESS_SYNCED} "
                                            f"{C.MESSAGE_RESOURCE_SYNCED.format('NexusAlgorithmTemplate')}"]
    # a complete set for this version whose flush finds the next version already cached (adopted, not yet
    # reported): nothing to do and nothing queued; the next version's reports bring the key back
    newer = env.cstate.update(R.TEMPLATES, NS, dict(new, spec=dict(spec, container=dict(spec["container"],
                                                                                         versionTag="v-3"))))
    ctl._on_crd_update(new, newer, C.KIND_TEMPLATE)
    assert ctl.stats["early_passes_skipped"] >= 1
    for i in range(2):
        ctl.on_executor_message(i, {"t": "report", "k": key, "u": new["metadata"]["uid"],
                                    "g": new["metadata"]["generation"], "r": {f"s{i}": None}, "w": True})
    env.refresh()  # the cache moves to `newer` before the batch is flushed
    ctl._inline_timer.cancel()
    ctl._flush_inline()
    assert ctl.stats["inline_superseded"] == 1 and len(ctl.queue) == 0 and ctl.queue.core.waiting() == 0
    events = len(env.recorder.events)
    report(newer["metadata"]["generation"])
    assert ctl.stats["inline_finishes"] == 2 and len(ctl.queue) == 0
    assert len(env.recorder.events) == events + 1  # the pending Synced Event went out with the newer version
    # a shard failure changes the status: queued
    report(newer["metadata"]["generation"], errs=(None, "ApiError: boom"))
    assert ctl.stats["inline_finishes"] == 2 and len(ctl.queue) == 1


async def test_status_patch_racing_a_spec_edit_drops_the_adoption_mark():
    """native status writes are merge PATCHes without a resourceVersion precondition, so the
    response can carry a user's spec edit made after our read.  If that edit adds a reference, the adoption
    mark must not move to the response's version: the next pass adopts the new Secret."""
    env = Env(1)
    t = env.seed()
    name, key = t["metadata"]["name"], make_key(C.KIND_TEMPLATE, NS, t["metadata"]["name"])
    ctl = env.build()
    await ctl.sync_template(NS, name)
    env.refresh()
    cur = ctl.template_lister.get(NS, name)
    assert ctl._adopted[key] == cur["metadata"]["resourceVersion"]
    env.cstate.create(R.SECRETS, NS, make_secret("s-new", NS))
    # the user adds a secretRef between our read and our status PATCH
    orig_patch = env.cclient.patch

    async def racing_patch(rt, ns, nm, body, **kw):
        if rt is R.TEMPLATES and kw.get("subresource") == "status":
            live = env.cstate.get(R.TEMPLATES, NS, name)
            spec = dict(live["spec"])
            rte = dict(spec["runtimeEnvironment"])
            rte["mappedEnvironmentVariables"] = list(rte["mappedEnvironmentVariables"]) + [
                {"secretRef": {"name": "s-new"}}]
            spec["runtimeEnvironment"] = rte
            env.cstate.update(R.TEMPLATES, NS, dict(live, spec=spec))
        return await orig_patch(rt, ns, nm, body, **kw)
    env.cclient.patch = racing_patch
    stale = dict(cur, status=dict(cur["status"], syncedToClusters=[]))  # forces a status write
    res = await ctl.report_template_synced_condition(stale, ["s"], ["c"], ["s0"])
    env.cclient.patch = orig_patch
    assert [e["secretRef"]["name"] for e in res["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"]
            if e.get("secretRef")] == ["s", "s-new"]
    assert ctl._adopted.get(key) != res["metadata"]["resourceVersion"]
    env.refresh()
    await ctl.sync_template(NS, name)
    owners = env.cstate.get(R.SECRETS, NS, "s-new")["metadata"].get("ownerReferences") or []
    assert [o["name"] for o in owners] == [name]


async def test_adoption_mark_not_stored_when_invalidated_during_adoption():
    """a dependent event that arrives while `adopt_references` is awaiting must win over the
    mark the pass would store afterwards."""
    env = Env(1)
    t = env.seed()
    name, key = t["metadata"]["name"], make_key(C.KIND_TEMPLATE, NS, t["metadata"]["name"])
    ctl = env.build()
    orig = ctl.adopt_references

    async def adopt_then_event(tpl):
        await orig(tpl)
        ctl._on_dependent(env.cstate.get(R.SECRETS, NS, "s"), "secret")  # e.g. our ownerRef removed
    ctl.adopt_references = adopt_then_event
    await ctl.sync_template(NS, name)
    assert key not in ctl._adopted


async def test_inline_finish_agrees_with_the_status_pass():
    """finish_inline's "status would not change" test is report_template_synced_condition's own decision."""
    env = Env(2)
    t = env.seed()
    ctl = env.build(role="coordinator")
    ctl.ready.set()
    name = t["metadata"]["name"]
    key = make_key(C.KIND_TEMPLATE, NS, name)
    base = ctl.template_lister.get(NS, name)
    good = {"conditions": [{"type": "Ready", "status": "True", "lastTransitionTime": "2026-01-01T00:00:00Z",
                            "reason": C.CONDITION_READY_REASON, "message": f'Algorithm "{name}" ready'}],
            "syncedSecrets": ["s"], "syncedConfigurations": ["c"], "syncedToClusters": ["s0", "s1"]}
    variants = [good, dict(good, syncedToClusters=["s0"]), dict(good, syncedSecrets=[]),
                {k: v for k, v in good.items() if k != "syncedConfigurations"},
                dict(good, conditions=[dict(good["conditions"][0], status="False")]),
                dict(good, conditions=[dict(good["conditions"][0], message="other")]),
                dict(good, conditions=good["conditions"] + [{"type": "Other"}]), dict(good, extra=1)]
    for st in variants:
        obj = dict(base, status=st)
        ctl.template_informer.store.upsert(obj)
        ctl._adopted[key] = obj["metadata"]["resourceVersion"]
        m = obj["metadata"]
        ctl.reports.feed(msgpack.packb({"t": "report", "k": key, "u": m["uid"], "g": int(m.get("generation") or 0),
                                        "r": {"s0": None, "s1": None}, "w": False}), False)
        old, new, _ = ctl._template_synced_status(obj, ["s"], ["c"], ["s0", "s1"])
        assert ctl.finish_inline(key) == (old == new), st
        assert ctl.finish_inline(key) == (old == new), st  # again: the memoised check agrees
    # the memo follows the shard list: a new list re-checks (and a status naming the old set needs a pass)
    obj = dict(base, status=good)
    ctl.template_informer.store.upsert(obj)
    ctl._adopted[key] = obj["metadata"]["resourceVersion"]
    assert ctl.finish_inline(key)
    ctl.all_shard_names = ["s0"]
    assert not ctl.finish_inline(key)


def test_coalescing_starts_only_inside_a_burst(monkeypatch):
    """Small batches and isolated changes are reconciled at once; only a run of more than BURST_MIN events,
    each less than one window after the previous, while BURST_MIN keys have work pending, is parked for the
    coalesce window.  Back-to-back small batches make a run but no load: no coalescing."""
    import ncc.controller.controller as ctl_mod
    env = Env(1)
    env.opts.coalesce_window = 0.002
    ctl = env.build()
    now = [100.0]
    monkeypatch.setattr(ctl_mod.time, "monotonic", lambda: now[0])

    def run(n):
        out = []
        for _ in range(n):
            now[0] += 0.0001
            out.append(ctl._coalesce_delay())
        return out
    assert run(ctl.BURST_MIN + 3) == [0.0] * (ctl.BURST_MIN + 3)  # a long run over an idle queue
    now[0] += 0.01  # a quiet window ends the run
    for i in range(ctl.BURST_MIN):
        ctl.queue.add(f"template/nexus/t{i}")
    delays = run(ctl.BURST_MIN + 3)
    assert delays[:ctl.BURST_MIN] == [0.0] * ctl.BURST_MIN and delays[ctl.BURST_MIN:] == [0.002] * 3
    now[0] += 0.01
    assert ctl._coalesce_delay() == 0.0


class _NoBatch:
    """The native report table without finish_batch: the controller takes the Python path."""

    def __init__(self, table):
        self._t = table

    def __getattr__(self, name):
        if name == "finish_batch":
            raise AttributeError(name)
        return getattr(self._t, name)


@pytest.mark.parametrize("native_queue", [False, True])
async def test_native_inline_finish_batch_matches_the_python_path(native_queue):
    """ReportTable.finish_batch decides exactly what `_finish_inline_py` decides, key by key: finished (with
    or without the Synced Event), a queued pass, superseded, or handed to the Python path (an overlaid object,
    a status not verified before) — same return value, memos, pending Events, stats and recorded Events."""
    import json as _json
    from ncc import native
    mod = native.load(required=True)
    good_status = lambda name: {  # noqa: E731
        "conditions": [{"type": "Ready", "status": "True", "lastTransitionTime": "2026-01-01T00:00:00Z",
                        "reason": C.CONDITION_READY_REASON, "message": f'Algorithm "{name}" ready'}],
        "syncedSecrets": ["s"], "syncedConfigurations": ["c"], "syncedToClusters": ["s0", "s1"]}

    def slim_template(i, status):
        t = make_template(i, NS, secrets=["s"], configmaps=["c"])
        t["metadata"].update(uid=f"u{i}", resourceVersion=str(100 + i), generation=2)
        t["status"] = status
        return mod.template_event_slim(_json.dumps({"type": "MODIFIED", "object": t}).encode())[1]

    def run(use_native):
        env = Env(2)
        env.opts.native_queue = native_queue
        ctl = env.build(role="coordinator")
        ctl.ready.set()
        if not use_native:
            ctl.reports = _NoBatch(ctl.reports)
        store = ctl.template_informer.store
        keys = []
        for i in range(11):
            name = make_template(i, NS)["metadata"]["name"]
            key = make_key(C.KIND_TEMPLATE, NS, name)
            keys.append(key)
            bad = i == 7
            obj = slim_template(i, dict(good_status(name), syncedToClusters=["s0"]) if bad else good_status(name))
            if i != 9:  # 9: not in the cache
                store.upsert(obj)
            if i != 4:  # 4: not adopted at this version
                ctl._adopted[key] = obj["metadata"]["resourceVersion"]
            if i not in (6, 7):  # 6, 7: this status not verified before
                ctl._inline_status_ok[key] = (obj["__ncc_sfp__"], obj["spec"]["_rfp"], ctl.all_shard_names)
            shards = {"s0": None} if i == 2 else {"s0": None, "s1": "boom" if i == 3 else None}
            ctl.reports.feed(msgpack.packb({"t": "report", "k": key, "u": f"u{i}", "g": 2, "r": shards,
                                            "w": False}), False)
            if i == 8:  # an overlaid (assumed) newer version
                store.assume(dict(obj, metadata=dict(obj["metadata"], resourceVersion=str(500 + i))))
        ctl._pending_event.update([keys[1], keys[6]])
        ctl.queue.add(keys[5])  # 5: a pass is queued
        keys.append(make_key(C.KIND_WORKGROUP, NS, "wg"))
        rest = ctl.finish_inline_many(keys)
        memo_keys = sorted(k for k in ctl._inline_status_ok)
        st = {k: ctl.stats[k] for k in ("reconciles", "inline_finishes", "inline_superseded")}
        return sorted(rest), memo_keys, sorted(ctl._pending_event), st, list(env.recorder.events)

    native_result, python_result = run(True), run(False)
    assert native_result == python_result
    rest, memos, pending, st, events = native_result
    # finished: 0, 1 (Event), 6 (verified now, Event), 10; superseded: 2; a pass: 3 (failure), 4 (not adopted),
    # 5 (busy), 7 (status needs a write), 8 (the overlaid version is not the adopted one), 9 (missing), workgroup
    assert st["inline_superseded"] == 1 and st["inline_finishes"] == 4 and len(events) == 2
    assert len(rest) == 7 and not pending
