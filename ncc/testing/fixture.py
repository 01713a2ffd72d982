"""Parity-test harness mirroring the reference's unit-test fixture (controller_test.go:50-797).

* one recording fake client for the controller cluster and one for a single shard ("shard0"),
  preloaded with `existing_*` objects (NewSimpleClientset(objects...));
* informers that are never started — their stores are seeded directly from `*_list_results`,
  so lister content and client content may differ on purpose, exactly as the reference seeds
  `Informer().GetIndexer()` (controller_test.go:546-576);
* a `FakeRecorder` that drops events (controller_test.go:544);
* sync handlers called directly; actions asserted per client *and API group* — the four
  client-go clientsets of the reference (controller-nexus, controller-kube, shard-nexus,
  shard-kube; controller_test.go:632-635) — in order, with condition `lastTransitionTime`
  normalised for status updates (controller_test.go:405-445).

Object builders reproduce `newTemplate`/`newSecret`/`newConfigMap`/`newWorkgroup`/`expected*`
(controller_test.go:151-379) as JSON-shaped dicts.
"""
from __future__ import annotations

from dataclasses import dataclass, field

from ..api import constants as C
from ..api import resources as R
from ..api.objects import deep_copy
from ..api.refs import ready_condition
from ..cache.informer import Informer
from ..controller.controller import Controller
from ..controller.events import FakeRecorder
from ..controller.options import ControllerOptions
from ..fakeapi.storage import ClusterState
from ..shards.shard import Shard
from .fake_client import Action, FakeClient

NS = "default"  # metav1.NamespaceDefault
ALIAS = "test-controller-cluster"
SHARD = "shard0"
CORE = "core"
NEXUS = C.GROUP


def expected_labels() -> dict:
    return C.owner_labels(ALIAS)


def owner_ref(t: dict) -> dict:
    return {"apiVersion": C.API_VERSION, "kind": C.TEMPLATE_KIND, "name": t["metadata"]["name"],
            "uid": t["metadata"].get("uid", "")}


def new_secret(name: str, owner: dict | None = None) -> dict:
    s = {"apiVersion": "v1", "kind": "Secret", "metadata": {"name": name, "namespace": NS}, "data": {}}
    if owner is not None:
        s["metadata"]["ownerReferences"] = [owner_ref(owner)]
    return s


def new_configmap(name: str, owner: dict | None = None) -> dict:
    c = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": name, "namespace": NS}, "data": {}}
    if owner is not None:
        c["metadata"]["ownerReferences"] = [owner_ref(owner)]
    return c


def new_template(name: str, secret: dict | None = None, configmap: dict | None = None, on_shard: bool = False,
                 status: dict | None = None) -> dict:
    env_from = [{}, {}]
    if secret is not None:
        env_from[0] = {"secretRef": {"name": secret["metadata"]["name"]}}
    if configmap is not None:
        env_from[1] = {"configMapRef": {"name": configmap["metadata"]["name"]}}
    t = {
        "apiVersion": C.API_VERSION,
        "kind": C.TEMPLATE_KIND,
        "metadata": {"name": name, "namespace": NS, "uid": name},
        "spec": {
            "container": {"image": "test", "registry": "test", "versionTag": "v1.0.0", "serviceAccountName": "test"},
            "computeResources": {"cpuLimit": "1000m", "memoryLimit": "2000Mi"},
            "workgroupRef": {"name": "test", "group": "test", "kind": "NexusAlgorithmWorkgroup"},
            "command": "python",
            "args": ["job.py"],
            "runtimeEnvironment": {"mappedEnvironmentVariables": env_from},
            "errorHandlingBehaviour": {"transientExitCodes": [], "fatalExitCodes": []},
            "datadogIntegrationSettings": {"mountDatadogSocket": True},
        },
    }
    if on_shard:
        t["metadata"]["labels"] = expected_labels()
    if status is not None:
        t["status"] = deep_copy(status)
    return t


def new_workgroup(name: str, on_shard: bool = False, cluster: str = SHARD, status: dict | None = None) -> dict:
    w = {
        "apiVersion": C.API_VERSION,
        "kind": C.WORKGROUP_KIND,
        "metadata": {"name": name, "namespace": NS, "uid": name},
        "spec": {"description": "test workgroup", "capabilities": {}, "cluster": cluster, "tolerations": [],
                 "affinity": {}},
    }
    if on_shard:
        w["metadata"]["labels"] = expected_labels()
    if status is not None:
        w["status"] = deep_copy(status)
    return w


def cond(status: bool, msg: str) -> dict:
    return ready_condition("2000-01-01T00:00:00Z", C.CONDITION_TRUE if status else C.CONDITION_FALSE, msg)


def expected_template(t: dict, secret: dict | None, configmap: dict | None, synced_to: list | None,
                      conditions: list | None) -> dict:
    out = deep_copy(t)
    st = out.setdefault("status", {})
    st["conditions"] = conditions
    if secret is not None:
        st["syncedSecrets"] = [secret["metadata"]["name"]]
    if configmap is not None:
        st["syncedConfigurations"] = [configmap["metadata"]["name"]]
    if synced_to is not None:
        st["syncedToClusters"] = synced_to
    return out


def expected_workgroup(w: dict, conditions: list) -> dict:
    out = deep_copy(w)
    out.setdefault("status", {})["conditions"] = conditions
    return out


def expected_shard_template(t: dict, uid: str) -> dict:
    out = deep_copy(t)
    out["metadata"]["uid"] = uid
    out["metadata"]["labels"] = expected_labels()
    out.pop("status", None)
    return out


def expected_shard_workgroup(w: dict, uid: str) -> dict:
    out = deep_copy(w)
    out["metadata"]["uid"] = uid
    out["metadata"]["labels"] = expected_labels()
    out.pop("status", None)
    return out


def expected_shard_dependent(src: dict, templates: list) -> dict:
    out = deep_copy(src)
    out["metadata"]["labels"] = expected_labels()
    out["metadata"]["ownerReferences"] = [owner_ref(t) for t in templates]
    return out


def canon(v):
    """Go omitempty view: drop None/""/{}/[] recursively (nil vs empty are indistinguishable in JSON)."""
    if isinstance(v, dict):
        out = {}
        for k, x in v.items():
            cx = canon(x)
            if cx is None or cx == "" or cx == {} or cx == []:
                continue
            out[k] = cx
        return out
    if isinstance(v, list):
        return [canon(x) for x in v]
    return v


def _norm_time(obj):
    obj = canon(obj)
    for c in (obj.get("status") or {}).get("conditions") or []:
        c["lastTransitionTime"] = "<t>"
    return obj


@dataclass
class Expect:
    verb: str
    rt: R.ResourceType
    obj: dict | None = None
    subresource: str = ""
    name: str = ""


@dataclass
class ClusterFixture:
    template_list: list = field(default_factory=list)
    workgroup_list: list = field(default_factory=list)
    secret_list: list = field(default_factory=list)
    configmap_list: list = field(default_factory=list)
    existing_core: list = field(default_factory=list)
    existing_nexus: list = field(default_factory=list)


class Fixture:
    def __init__(self, controller: ClusterFixture | None = None, shard: ClusterFixture | None = None,
                 options: ControllerOptions | None = None):
        self.cf = controller or ClusterFixture()
        self.sf = shard or ClusterFixture()
        self.options = options or ControllerOptions.compat(native_queue=False)
        self.expect: dict[tuple[str, str], list[Expect]] = {("controller", NEXUS): [], ("controller", CORE): [],
                                                            ("shard", NEXUS): [], ("shard", CORE): []}

    def new_controller(self) -> Controller:
        self.controller_client = FakeClient(ClusterState("controller", simple=True), cluster_name="controller")
        self.shard_client = FakeClient(ClusterState(SHARD, simple=True), cluster_name=SHARD)
        for o in self.cf.existing_core + self.cf.existing_nexus:
            self.controller_client.seed(R.by_kind(o["kind"]), o)
        for o in self.sf.existing_core + self.sf.existing_nexus:
            self.shard_client.seed(R.by_kind(o["kind"]), o)
        cc = self.controller_client
        infs = {rt: Informer(cc, rt, None) for rt in (R.TEMPLATES, R.WORKGROUPS, R.SECRETS, R.CONFIGMAPS)}
        shard = Shard(ALIAS, SHARD, self.shard_client, None)
        for o in self.cf.template_list:
            infs[R.TEMPLATES].store.upsert(o)
        for o in self.cf.workgroup_list:
            infs[R.WORKGROUPS].store.upsert(o)
        for o in self.cf.secret_list:
            infs[R.SECRETS].store.upsert(o)
        for o in self.cf.configmap_list:
            infs[R.CONFIGMAPS].store.upsert(o)
        for o in self.sf.template_list:
            shard.template_informer.store.upsert(o)
        for o in self.sf.workgroup_list:
            shard.workgroup_informer.store.upsert(o)
        for o in self.sf.secret_list:
            shard.secret_informer.store.upsert(o)
        for o in self.sf.configmap_list:
            shard.configmap_informer.store.upsert(o)
        self.recorder = FakeRecorder(keep=True)
        self.controller = Controller(alias=ALIAS, namespace="test", client=cc, shards=[shard],
                                     template_informer=infs[R.TEMPLATES], workgroup_informer=infs[R.WORKGROUPS],
                                     secret_informer=infs[R.SECRETS], configmap_informer=infs[R.CONFIGMAPS],
                                     options=self.options, recorder=self.recorder)
        self.shard = shard
        return self.controller

    # ---------------------------------------------------------------- expectations
    def expect_controller_status(self, obj: dict, rt=R.TEMPLATES) -> None:
        self.expect[("controller", NEXUS)].append(Expect("update", rt, obj, "status"))

    def expect_controller_update(self, obj: dict) -> None:
        self.expect[("controller", CORE)].append(Expect("update", R.by_kind(obj["kind"]), obj))

    def expect_shard(self, verb: str, obj: dict, rt: R.ResourceType | None = None) -> None:
        rt = rt or R.by_kind(obj["kind"])
        self.expect[("shard", rt.group_key)].append(Expect(verb, rt, obj, name=obj["metadata"]["name"]))

    # ---------------------------------------------------------------- run + check
    async def run(self, templates: list = (), workgroups: list = (), expect_error: bool = False) -> list:
        c = self.new_controller()
        errors = []
        for ns, name in templates:
            try:
                await c.sync_template(ns, name)
                if expect_error:
                    errors.append("expected error syncing template, got nil")
            except Exception as e:  # noqa: BLE001
                if not expect_error:
                    errors.append(f"error syncing template: {e!r}")
        for ns, name in workgroups:
            try:
                await c.sync_workgroup(ns, name)
                if expect_error:
                    errors.append("expected error syncing workgroup, got nil")
            except Exception as e:  # noqa: BLE001
                if not expect_error:
                    errors.append(f"error syncing workgroup: {e!r}")
        errors += self.check(("controller", NEXUS), self.controller_client.actions)
        errors += self.check(("shard", NEXUS), self.shard_client.actions)
        errors += self.check(("shard", CORE), self.shard_client.actions)
        errors += self.check(("controller", CORE), self.controller_client.actions)
        return errors

    async def run_object_handler(self, objs: list) -> list:
        import inspect
        c = self.new_controller()
        for o in objs:
            r = c.handle_object(o)
            if inspect.isawaitable(r):
                await r
        errors = self.check(("shard", NEXUS), self.shard_client.actions)
        errors += self.check(("shard", CORE), self.shard_client.actions)
        return errors

    def check(self, which: tuple, actions: list[Action]) -> list:
        _, group = which
        acts = [a for a in actions if a.group == group and a.verb not in ("list", "watch", "get")]
        exp = self.expect[which]
        errs = []
        for i, a in enumerate(acts):
            if i >= len(exp):
                errs.append(f"{which}: {len(acts) - len(exp)} unexpected actions: {acts[i:]}")
                break
            e = exp[i]
            if e.verb != a.verb or e.rt.plural != a.resource.plural or e.subresource != a.subresource:
                errs.append(f"{which}[{i}]: expected {e.verb} {e.rt.plural}/{e.subresource}, got {a!r}")
                continue
            if a.verb == "delete":
                if e.name != a.name:
                    errs.append(f"{which}[{i}]: delete targets {a.name}, expected {e.name}")
                continue
            want = _norm_time(e.obj) if a.verb == "update" else canon(e.obj)
            got = _norm_time(a.obj) if a.verb == "update" else canon(a.obj)
            if want != got:
                errs.append(f"{which}[{i}] {a.verb} {a.resource.plural} has wrong object\n want={want}\n  got={got}")
        if len(exp) > len(acts):
            errs.append(f"{which}: {len(exp) - len(acts)} additional expected actions: {exp[len(acts):]}")
        return errs
