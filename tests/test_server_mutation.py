"""Shards whose apiserver stores something other than what the controller sent.

CRD structural defaulting/pruning (a shard running another NexusAlgorithmTemplate CRD) and a mutating
admission webhook (ncc/fakeapi/admission.py) rewrite the controller's shard writes.  Native mode caches
its own writes (slim caches publish the request body, watch echoes are promoted undecoded —
ncc/shards/shard.py `_tracked`, ncc/cache/informer.py `end_write`), so these tests pin that:

* the caches see the stored (mutated) state, not the request body;
* there is no write loop — once converged, a quiet window has no shard writes at all;
* drift made by someone else is still repaired (the "our write produced this version" mark never hides
  a later version), and controller-side changes still propagate;
* Ready is reported only once the shard holds the controller's content (as mutated by the server).

The reference compares typed objects with reflect.DeepEqual (controller.go:539,600,725,795): on such a
shard it issues a no-op update on every pass; compat mode keeps that behaviour.
"""
import asyncio
import copy

import pytest

from ncc.api import constants as C
from ncc.api import resources as R
from ncc.api.fingerprint import SLIM_FP, SLIM_WROTE, fingerprint
from ncc.api.schema import default_and_prune, default_and_prune_object
from ncc.fakeapi.admission import Admission
from test_e2e import NS, Running, mutate, wait_for
from ncc.testing.env import FakeEnvironment
from ncc.testing.workload import make_configmap, make_secret, make_template

INJECTED = "aW5qZWN0ZWQ="  # base64("injected")


def _older_template_crd(crd: dict) -> dict:
    """The shard's CRD: spec.container.pullPolicy defaults to IfNotPresent, and spec neither knows nor
    preserves datadogIntegrationSettings (pruned)."""
    crd = copy.deepcopy(crd)
    v = crd["spec"]["versions"][0]["schema"]["openAPIV3Schema"]
    spec = v["properties"]["spec"]
    spec["x-kubernetes-preserve-unknown-fields"] = False
    spec["properties"].pop("datadogIntegrationSettings")
    spec["properties"]["container"]["properties"]["pullPolicy"] = {"type": "string", "default": "IfNotPresent"}
    return crd


def _mutating_shard(env: FakeEnvironment) -> None:
    st = env.shard_servers[0].state
    key = (C.GROUP, R.TEMPLATES.plural)
    st.crds[key] = _older_template_crd(st.crds[key])
    st.admission.update({"prune_defaults": True,
                         "sets": {"secrets": {"data.injected": INJECTED},
                                  "configmaps": {"data.injected": "yes"}}})


def _shard_writes(env: FakeEnvironment) -> int:
    s = env.shard_servers[0].state.stats
    return s["create"] + s["update"] + s["patch"] + s["noop_update"]


async def _quiet(env: FakeEnvironment, window: float = 1.0, timeout: float = 10.0) -> int:
    """Wait for a `window` without any shard write (no write loop); returns the writes so far.  Compat mode
    (5 QPS client, one no-op shard update per pass, as the reference) takes a few seconds to get there."""
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    while True:
        before = _shard_writes(env)
        await asyncio.sleep(window)
        if _shard_writes(env) == before:
            return before
        assert loop.time() < end, f"shard writes never stop: {env.shard_servers[0].state.stats}"


async def _ready(cc, name):
    o = await cc.get(R.TEMPLATES, NS, name)
    conds = (o.get("status") or {}).get("conditions") or []
    return bool(conds) and conds[0]["status"] == "True"


CASES = [
    pytest.param("compat", {}, id="compat"),
    pytest.param("native", {"executors": 0}, id="native-inprocess"),
    pytest.param("native", {"executor_impl": "python"}, id="native-python-executor"),
    pytest.param("native", {"executor_impl": "native"}, id="native-cpp-executor"),
]


@pytest.mark.parametrize("mode,cfg", CASES)
async def test_server_side_mutation_no_loop_no_false_ready(tmp_path, mode, cfg):
    if cfg.get("executor_impl") == "native":
        from ncc.controller.native_executor import binary_path
        if binary_path() is None:
            pytest.skip("ncc/bin/ncc-executor not built")
    env = await FakeEnvironment(1, str(tmp_path)).start()
    _mutating_shard(env)
    cc, sc = env.controller_client(), env.shard_client(0)
    try:
        await cc.create(R.SECRETS, NS, make_secret("s0", NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap("c0", NS))
        for i in range(2):
            await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=["s0"], configmaps=["c0"]))
        src_secret = await cc.get(R.SECRETS, NS, "s0")
        async with Running(env, mode, **cfg) as app:
            for i in range(2):
                await wait_for(lambda i=i: _ready(cc, f"algo-{i:05d}"), timeout=5)
            # the shard holds the controller's content as its apiserver rewrote it
            st = await sc.get(R.TEMPLATES, NS, "algo-00000")
            assert st["spec"]["container"]["pullPolicy"] == "IfNotPresent"
            assert "datadogIntegrationSettings" not in st["spec"]
            sec = await sc.get(R.SECRETS, NS, "s0")
            assert sec["data"] == dict(src_secret["data"], injected=INJECTED)
            cm = await sc.get(R.CONFIGMAPS, NS, "c0")
            assert cm["data"]["injected"] == "yes"

            # no write loop: after convergence a quiet window sees no shard write at all
            settled = await _quiet(env)
            if mode == "native":  # 6 objects: a create each, at most one re-write of a mutated version each
                assert settled <= 12, env.shard_servers[0].state.stats

            if cfg.get("executors") == 0:
                # the in-process caches hold what the server stored (not the request body), marked with
                # the digest of what was sent
                shard = app.controller.shards[0]
                cached = shard.secret_informer.store.get(NS, "s0")
                assert cached[SLIM_FP][0] == fingerprint(sec["data"])
                assert cached[SLIM_WROTE][0] == fingerprint(src_secret["data"])
                ct = shard.template_informer.store.get(NS, "algo-00000")
                assert ct[SLIM_FP][0] == fingerprint(st["spec"])
                assert shard.server_rewrites >= 3

            # drift by someone else on a mutated object is still repaired
            await mutate(sc, R.SECRETS, "s0", lambda o: o["data"].__setitem__("token", "dGFtcGVyZWQ="))
            await mutate(sc, R.TEMPLATES, "algo-00001",
                         lambda o: o["spec"]["container"].__setitem__("versionTag", "tampered"))

            async def repaired():
                s = await sc.get(R.SECRETS, NS, "s0")
                t = await sc.get(R.TEMPLATES, NS, "algo-00001")
                return s["data"]["token"] == src_secret["data"]["token"] and \
                    t["spec"]["container"]["versionTag"] == "v1.0.0"
            if mode == "native":  # compat repairs shard drift only on the next controller-side event/resync
                await wait_for(repaired, timeout=5)

            # controller-side changes propagate (and are mutated again), and Ready follows the shard content
            await mutate(cc, R.SECRETS, "s0", lambda o: o["data"].__setitem__("token", "bmV3"))
            await mutate(cc, R.TEMPLATES, "algo-00000",
                         lambda o: o["spec"]["container"].__setitem__("versionTag", "v2.0.0"))

            async def propagated():
                s = await sc.get(R.SECRETS, NS, "s0")
                t = await sc.get(R.TEMPLATES, NS, "algo-00000")
                return s["data"]["token"] == "bmV3" and s["data"]["injected"] == INJECTED and \
                    t["spec"]["container"]["versionTag"] == "v2.0.0" and \
                    t["spec"]["container"]["pullPolicy"] == "IfNotPresent"
            await wait_for(propagated, timeout=5)
            await wait_for(lambda: _ready(cc, "algo-00000"), timeout=5)
            await _quiet(env)
    finally:
        await cc.close()
        await sc.close()
        await env.stop()


def test_default_and_prune():
    s = {"type": "object", "properties": {
        "a": {"type": "object", "properties": {"x": {"type": "string", "default": "d"}}},
        "keep": {"type": "object", "x-kubernetes-preserve-unknown-fields": True},
        "m": {"type": "object", "additionalProperties": {"type": "object", "properties": {"y": {"type": "integer"}}}},
        "l": {"type": "array", "items": {"type": "object", "properties": {"z": {"type": "string"}}}},
        "d": {"type": "object", "default": {}, "properties": {"w": {"type": "integer", "default": 3}}}}}
    v = {"a": {}, "junk": 1, "keep": {"any": [1]}, "m": {"k": {"y": 1, "q": 2}}, "l": [{"z": "1", "r": 0}]}
    assert default_and_prune(s, v) == {"a": {"x": "d"}, "keep": {"any": [1]}, "m": {"k": {"y": 1}},
                                       "l": [{"z": "1"}], "d": {"w": 3}}
    crd = {"spec": {"versions": [{"name": "v1", "schema": {"openAPIV3Schema": {
        "type": "object", "properties": {"spec": s}}}}]}}
    obj = {"apiVersion": "g/v1", "kind": "K", "metadata": {"name": "n"}, "spec": {"junk": 1}, "other": 2}
    assert default_and_prune_object(crd, obj, "v1") == {"apiVersion": "g/v1", "kind": "K",
                                                        "metadata": {"name": "n"}, "spec": {"d": {"w": 3}}}


def test_admission_sets():
    a = Admission()
    assert not a.active
    a.update({"sets": {"secrets": {"data.injected": "x", "metadata.labels.team": "a", "type": None}}})
    o = {"metadata": {"name": "s"}, "type": "Opaque"}
    a.admit(R.SECRETS, o, None)
    assert o == {"metadata": {"name": "s", "labels": {"team": "a"}}, "data": {"injected": "x"}}
    assert a.mutated == 1
    a.admit(R.SECRETS, o, None)  # already as the webhook wants it
    assert a.mutated == 1
    o2 = {"metadata": {"name": "c"}}
    a.admit(R.CONFIGMAPS, o2, None)
    assert o2 == {"metadata": {"name": "c"}}
    a.admit(R.SECRETS, o2, None, subresource="status")  # webhooks here only see the main resource
    assert o2 == {"metadata": {"name": "c"}}


def test_members_equal():
    from ncc import native
    m = native.load()
    if m is None:
        pytest.skip("native extension not built")
    assert m.members_equal(b'{"a":1,"spec":{"x":[1,"}"]}}', b'{"metadata":{},"spec":{"x":[1,"}"]}}', ("spec", "data"))
    assert not m.members_equal(b'{"spec":{"x":1}}', b'{"spec":{"x": 1}}', ("spec",))  # bytes, not JSON equality
    assert not m.members_equal(b'{"data":{}}', b'{}', ("data",))
    assert m.members_equal(b'{}', b'{"other":1}', ("data",))
    assert not m.members_equal(b'not json', b'{}', ("data",))
    assert not m.members_equal(b'{"da\\u0074a":1}', b'{"data":1}', ("data",))  # escaped keys: decode instead
