"""Against real clusters: the reference's `Test_ControllerMain` (controller_test.go:1287-1336).

Skipped unless `NEXUS__CONTROLLER_CONFIG_PATH` (controller kubeconfig) and `NEXUS__SHARD_CONFIG_PATH`
(directory of `<shard>.kubeconfig` files) point at live kube-apiservers with the Nexus CRDs installed
(deploy/crds) and the `nexus` namespace present — the `kind-e2e` job of .github/workflows/ci.yaml creates
exactly that with two kind clusters, as the reference's build.yaml:44-80 does.  Everything else in the
suite runs against ncc/fakeapi; this is where real-apiserver behaviour (defaulting, managedFields,
strategic merge, watch bookmarks, RBAC) is exercised.

`python -m ncc` runs as a child process with the caller's NEXUS__* environment (mode from
NCC_LIVE_MODES, default "native,compat"), like the reference's `go main()`.  Steps, each with the
reference's 1 s budget stretched to NCC_LIVE_STEP_S (default 10 s) for slower CI runners:
create → shard copy (+ Secret/ConfigMap with the shard template as owner) → versionTag update propagates →
Ready condition → delete propagates.  Objects are namespaced by a random suffix and cleaned up.
"""
import asyncio
import os
import subprocess
import sys
import uuid

import pytest

from ncc.api import constants as C
from ncc.api import resources as R
from ncc.kube import errors as E
from ncc.kube.kubeconfig import load_kubeconfig
from ncc.kube.rest import RestClient
from ncc.testing.workload import make_configmap, make_secret, make_template

CTRL = os.environ.get("NEXUS__CONTROLLER_CONFIG_PATH", "")
SHARDS = os.environ.get("NEXUS__SHARD_CONFIG_PATH", "")
NS = os.environ.get("NEXUS__CONTROLLER_NAMESPACE", "nexus")
STEP_S = float(os.environ.get("NCC_LIVE_STEP_S", "10"))
MODES = [m for m in os.environ.get("NCC_LIVE_MODES", "native,compat").split(",") if m]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _shard_kubeconfigs() -> list:
    if not SHARDS or not os.path.isdir(SHARDS):
        return []
    return sorted(os.path.join(SHARDS, f) for f in os.listdir(SHARDS) if not f.startswith("."))


pytestmark = pytest.mark.skipif(not (CTRL and os.path.isfile(CTRL) and _shard_kubeconfigs()),
                                reason="live clusters not configured (NEXUS__CONTROLLER_CONFIG_PATH / "
                                       "NEXUS__SHARD_CONFIG_PATH)")


async def _eventually(fn, what: str, timeout: float = STEP_S):
    loop = asyncio.get_running_loop()
    end = loop.time() + timeout
    last = None
    while loop.time() < end:
        try:
            last = await fn()
            if last:
                return last
        except E.NotFound as e:
            last = e
        await asyncio.sleep(0.1)
    raise AssertionError(f"{what}: not within {timeout}s (last: {last!r})")


async def _gone(client, rt, name):
    try:
        await client.get(rt, NS, name)
        return False
    except E.NotFound:
        return True


@pytest.mark.parametrize("mode", MODES)
async def test_controller_main_against_live_clusters(mode, tmp_path):
    suffix = uuid.uuid4().hex[:6]
    tname, sname, cname = f"ncc-live-{suffix}", f"ncc-live-s-{suffix}", f"ncc-live-c-{suffix}"
    cc = RestClient(load_kubeconfig(CTRL, name="controller"))
    scs = [RestClient(load_kubeconfig(p, name=os.path.basename(p))) for p in _shard_kubeconfigs()]
    env = dict(os.environ, NEXUS__MODE=mode, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    env.setdefault("NEXUS__ALIAS", "kind-nexus-controller")
    log = open(tmp_path / "controller.log", "wb")
    proc = None
    try:
        await cc.create(R.SECRETS, NS, make_secret(sname, NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap(cname, NS))
        t = make_template(0, NS, secrets=[sname], configmaps=[cname])
        t["metadata"]["name"] = tname
        await cc.create(R.TEMPLATES, NS, t)
        proc = subprocess.Popen([sys.executable, "-m", "ncc"], env=env, stdout=log, stderr=subprocess.STDOUT)

        for sc in scs:  # template, then its dependents owned by the shard template
            st = await _eventually(lambda sc=sc: sc.get(R.TEMPLATES, NS, tname), "shard template")
            assert st["metadata"]["labels"][C.LABEL_CONFIGURATION_OWNER] == env["NEXUS__ALIAS"]
            for rt, n in ((R.SECRETS, sname), (R.CONFIGMAPS, cname)):
                dep = await _eventually(lambda sc=sc, rt=rt, n=n: sc.get(rt, NS, n), f"shard {rt.kind}")
                assert [r["uid"] for r in dep["metadata"]["ownerReferences"]] == [st["metadata"]["uid"]]

        cur = await cc.get(R.TEMPLATES, NS, tname)
        cur["spec"]["container"]["versionTag"] = "v2.3.4"
        await cc.update(R.TEMPLATES, NS, cur)
        for sc in scs:
            async def updated(sc=sc):
                o = await sc.get(R.TEMPLATES, NS, tname)
                return o["spec"]["container"]["versionTag"] == "v2.3.4"
            await _eventually(updated, "versionTag update on the shard")

        async def ready():
            o = await cc.get(R.TEMPLATES, NS, tname)
            conds = (o.get("status") or {}).get("conditions") or []
            return bool(conds) and conds[0]["status"] == "True" and \
                len(o["status"].get("syncedToClusters") or []) == len(scs)
        await _eventually(ready, "Ready condition")

        await cc.delete(R.TEMPLATES, NS, tname)
        for sc in scs:
            await _eventually(lambda sc=sc: _gone(sc, R.TEMPLATES, tname), "shard template deletion")
        assert proc.poll() is None, "controller exited"
    finally:
        if proc is not None:
            proc.terminate()
            try:
                proc.wait(timeout=20)
            except subprocess.TimeoutExpired:
                proc.kill()
        log.close()
        for client in [cc] + scs:
            for rt, n in ((R.TEMPLATES, tname), (R.SECRETS, sname), (R.CONFIGMAPS, cname)):
                try:
                    await client.delete(rt, NS, n)
                except E.ApiError:
                    pass
            await client.close()
