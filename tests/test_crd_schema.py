"""The shipped CRDs (deploy/crds, also bundled in the Helm chart) as a contract: every object shape the
reference's tests use validates, the controller's status writes validate (the e2e apiservers enforce
it), and the fake apiserver rejects schema violations with 422 Invalid like a real one."""
import filecmp
import os

import pytest

from ncc.api import resources as R
from ncc.api.refs import ready_condition
from ncc.api.schema import load_crds, validate, validate_object
from ncc.kube import errors as E
from ncc.testing.env import FakeEnvironment
from ncc.testing.workload import make_template, make_workgroup

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRDS = load_crds(os.path.join(ROOT, "deploy", "crds"))
TPL = CRDS[("science.sneaksanddata.com", "nexusalgorithmtemplates")]
WG = CRDS[("science.sneaksanddata.com", "nexusalgorithmworkgroups")]


def test_helm_chart_bundles_the_same_crds():
    a, b = os.path.join(ROOT, "deploy", "crds"), os.path.join(ROOT, "deploy", "helm",
                                                              "nexus-configuration-controller", "crds")
    names = sorted(os.listdir(a))
    assert names == sorted(os.listdir(b))
    assert all(filecmp.cmp(os.path.join(a, n), os.path.join(b, n), shallow=False) for n in names)


def test_reference_object_shapes_validate():
    # controller_test.go:230-333 builds templates with every spec section; make_template mirrors it
    t = make_template(3, "nexus", secrets=["s1", "s2"], configmaps=["c1"])
    t["status"] = {"conditions": [ready_condition("2025-09-19T00:00:00Z", "True", 'Algorithm "x" ready')],
                   "syncedSecrets": ["s1", "s2"], "syncedConfigurations": ["c1"], "syncedToClusters": ["shard0"]}
    assert validate_object(TPL, t) == []
    w = make_workgroup("mi355x", "nexus")
    w["status"] = {"conditions": [ready_condition("2025-09-19T00:00:00Z", "False", 'Workgroup "w" initializing')]}
    assert validate_object(WG, w) == []


def test_schema_violations_are_reported():
    t = make_template(0, "nexus")
    t["spec"]["args"] = "not-a-list"
    t["spec"]["runtimeEnvironment"]["deadlineSeconds"] = 2 ** 40
    t["status"] = {"conditions": [{"type": "Ready", "status": "Maybe"}], "syncedToClusters": [1]}
    errs = validate_object(TPL, t)
    assert "spec.args: Invalid value: str: must be of type array" in errs
    assert any(e.startswith("spec.runtimeEnvironment.deadlineSeconds: Invalid value") for e in errs)
    assert "status.conditions[0].reason: Required value" in errs
    assert any(e.startswith("status.conditions[0].status: Unsupported value") for e in errs)
    assert "status.syncedToClusters[0]: Invalid value: int: must be of type string" in errs
    # unknown spec fields survive (x-kubernetes-preserve-unknown-fields), unknown status fields do not
    t2 = make_template(0, "nexus")
    t2["spec"]["somethingNewInNexusCore"] = {"a": 1}
    t2["status"] = {"observedBy": "x"}
    assert validate_object(TPL, t2) == ["status.observedBy: Unknown field"]
    assert validate({"type": "integer", "nullable": True}, None) == []
    assert validate({"type": "object", "additionalProperties": False}, {"x": 1}) == ["x: Unknown field"]


async def test_fake_apiserver_rejects_invalid_custom_resources(tmp_path):
    env = await FakeEnvironment(0, str(tmp_path)).start()
    cc = env.controller_client()
    try:
        t = make_template(0, "nexus")
        t["spec"]["args"] = 42
        with pytest.raises(E.Invalid) as ei:
            await cc.create(R.TEMPLATES, "nexus", t)
        assert "spec.args" in str(ei.value)
        ok = await cc.create(R.TEMPLATES, "nexus", make_template(1, "nexus"))
        bad = dict(ok, status={"conditions": [{"type": "Ready", "status": "True"}]})
        with pytest.raises(E.Invalid):
            await cc.update_status(R.TEMPLATES, "nexus", bad)
        good = dict(ok, status={"conditions": [ready_condition("2025-09-19T00:00:00Z", "True", "ready")]})
        assert (await cc.update_status(R.TEMPLATES, "nexus", good))["status"]["conditions"][0]["status"] == "True"
    finally:
        await cc.close()
        await env.stop()
