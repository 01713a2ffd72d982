"""Reference parity: the ten unit tests of controller_test.go:800-1285, action-for-action.

Each test builds the same controller/shard fixtures as the Go test, runs the same sync handler,
and asserts the same ordered per-client write actions (SURVEY.md §4 test matrix), in
reference-compat mode.
"""
from ncc.api import resources as R
from ncc.api.objects import deep_copy
from ncc.testing.fixture import (NS, ClusterFixture, Fixture, cond, expected_shard_dependent,
                                 expected_shard_template, expected_shard_workgroup, expected_template,
                                 expected_workgroup, new_configmap, new_secret, new_template, new_workgroup,
                                 owner_ref)


def provision():
    s, c = new_secret("test-secret"), new_configmap("test-config")
    return s, c, new_template("test", s, c)


def owned(s, c, t):
    so, co = deep_copy(s), deep_copy(c)
    so["metadata"]["ownerReferences"] = [owner_ref(t)]
    co["metadata"]["ownerReferences"] = [owner_ref(t)]
    return so, co


def ref(o):
    return (o["metadata"]["namespace"], o["metadata"]["name"])


async def test_creates_template():
    s, c, t = provision()
    so, co = owned(s, c, t)
    f = Fixture(ClusterFixture(template_list=[t], secret_list=[s], configmap_list=[c], existing_core=[s, c],
                               existing_nexus=[t]))
    f.expect_controller_status(expected_template(t, None, None, None, [cond(False, 'Algorithm "test" initializing')]))
    f.expect_controller_status(expected_template(t, s, c, ["shard0"], [cond(True, 'Algorithm "test" ready')]))
    f.expect_controller_update(so)
    f.expect_controller_update(co)
    st = expected_shard_template(t, "")
    f.expect_shard("create", st)
    f.expect_shard("create", expected_shard_dependent(s, [st]))
    f.expect_shard("create", expected_shard_dependent(c, [st]))
    errs = await f.run(templates=[ref(t)])
    assert not errs, "\n".join(errs)
    assert f.recorder.events == ["Normal Synced Resource of type NexusAlgorithmTemplate synced successfully"]


async def test_detects_rogue():
    s, c, t = provision()
    so, co = owned(s, c, t)
    f = Fixture(ClusterFixture(template_list=[t], secret_list=[s], configmap_list=[c], existing_core=[s, c],
                               existing_nexus=[t]),
                ClusterFixture(secret_list=[s]))
    f.expect_controller_status(expected_template(t, None, None, None, [cond(False, 'Algorithm "test" initializing')]))
    f.expect_shard("create", expected_shard_template(t, ""))  # then fail-fast on the rogue secret
    f.expect_controller_update(so)
    f.expect_controller_update(co)
    errs = await f.run(templates=[ref(t)], expect_error=True)
    assert not errs, "\n".join(errs)
    assert any("ErrResourceExists" in e and 'Resource "test-secret" already exists' in e for e in f.recorder.events)
    assert any("ErrResourceSyncError" in e for e in f.recorder.events)


async def test_handles_not_existing_resource():
    _, _, t = provision()
    f = Fixture(ClusterFixture())
    errs = await f.run(templates=[ref(t)])
    assert not errs, "\n".join(errs)


async def test_skips_invalid_template():
    _, _, t = provision()
    f = Fixture(ClusterFixture(template_list=[t], existing_nexus=[t]))
    f.expect_controller_status(expected_template(t, None, None, None, [cond(False, 'Algorithm "test" initializing')]))
    errs = await f.run(templates=[ref(t)], expect_error=True)
    assert not errs, "\n".join(errs)
    assert f.recorder.events == ['Warning ErrResourceMissing Resource "test-secret" referenced by NexusAlgorithmTemplate '
                                 '"test" is missing in the controller cluster']


async def test_updates_template_secret_and_config():
    s, c, t0 = provision()
    so, co = owned(s, c, t0)
    s_upd = deep_copy(so)
    s_upd["data"] = {"secret.file": "dXBkYXRlZC1zZWNyZXQ="}  # []byte("updated-secret")
    c_upd = deep_copy(co)
    c_upd["data"] = {"new.file": "updated-config"}
    t = new_template("test", s_upd, c_upd, status={
        "syncedSecrets": ["test-secret"], "syncedConfigurations": ["test-config"], "syncedToClusters": ["shard0"],
        "conditions": [cond(True, 'Algorithm "test" ready')]})
    t_shard = new_template("test", s, c, on_shard=True)
    s_shard = new_secret("test-secret", t_shard)
    s_shard_upd = deep_copy(s_shard)
    s_shard_upd["data"] = dict(s_upd["data"])
    c_shard = new_configmap("test-config", t_shard)
    c_shard_upd = deep_copy(c_shard)
    c_shard_upd["data"] = dict(c_upd["data"])
    f = Fixture(ClusterFixture(template_list=[t], secret_list=[s_upd], configmap_list=[c_upd],
                               existing_core=[s_upd, c_upd], existing_nexus=[t]),
                ClusterFixture(template_list=[t_shard], secret_list=[s_shard], configmap_list=[c_shard],
                               existing_core=[s_shard, c_shard], existing_nexus=[t_shard]))
    f.expect_shard("update", s_shard_upd)
    f.expect_shard("update", c_shard_upd)
    errs = await f.run(templates=[ref(t)])
    assert not errs, "\n".join(errs)


async def test_creates_shared_resources():
    s, c = new_secret("test-secret"), new_configmap("test-config")
    t1 = new_template("test1", s, c, status={
        "syncedSecrets": ["test-secret"], "syncedConfigurations": ["test-config"], "syncedToClusters": ["shard0"],
        "conditions": [cond(True, 'Algorithm "test1" ready')]})
    so1, co1 = owned(s, c, t1)
    t2 = new_template("test2", s, c)
    so12, co12 = deep_copy(so1), deep_copy(co1)
    so12["metadata"]["ownerReferences"].append(owner_ref(t2))
    co12["metadata"]["ownerReferences"].append(owner_ref(t2))
    t1_shard = expected_shard_template(t1, "test1")
    s_shard1 = expected_shard_dependent(s, [t1_shard])
    c_shard1 = expected_shard_dependent(c, [t1_shard])
    t1_ctrl = expected_template(t1, s, c, ["shard0"], [cond(True, 'Algorithm "test1" ready')])
    f = Fixture(ClusterFixture(template_list=[t1_ctrl, t2], secret_list=[so1], configmap_list=[co1],
                               existing_core=[so1, co1], existing_nexus=[t1_ctrl, t2]),
                ClusterFixture(template_list=[t1_shard], secret_list=[s_shard1], configmap_list=[c_shard1],
                               existing_core=[s_shard1, c_shard1], existing_nexus=[t1_shard]))
    f.expect_controller_status(expected_template(t2, None, None, None,
                                                 [cond(False, 'Algorithm "test2" initializing')]))
    f.expect_controller_status(expected_template(t2, s, c, ["shard0"], [cond(True, 'Algorithm "test2" ready')]))
    f.expect_controller_update(so12)
    f.expect_controller_update(co12)
    t2_shard = expected_shard_template(t2, "")
    f.expect_shard("create", t2_shard)
    f.expect_shard("update", expected_shard_dependent(s_shard1, [t1_shard, t2_shard]))
    f.expect_shard("update", expected_shard_dependent(c_shard1, [t1_shard, t2_shard]))
    errs = await f.run(templates=[ref(t2)])
    assert not errs, "\n".join(errs)


async def test_takes_ownership():
    s, c, t = provision()
    so, co = owned(s, c, t)
    rogue = expected_shard_template(t, "")
    rogue["spec"]["datadogIntegrationSettings"]["mountDatadogSocket"] = False
    f = Fixture(ClusterFixture(template_list=[t], secret_list=[s], configmap_list=[c], existing_core=[s, c],
                               existing_nexus=[t]),
                ClusterFixture(template_list=[rogue], existing_nexus=[rogue]))
    f.expect_controller_status(expected_template(t, None, None, None, [cond(False, 'Algorithm "test" initializing')]))
    f.expect_controller_status(expected_template(t, s, c, ["shard0"], [cond(True, 'Algorithm "test" ready')]))
    f.expect_controller_update(so)
    f.expect_controller_update(co)
    st = expected_shard_template(t, "")
    f.expect_shard("update", st)
    f.expect_shard("create", expected_shard_dependent(s, [st]))
    f.expect_shard("create", expected_shard_dependent(c, [st]))
    errs = await f.run(templates=[ref(t)])
    assert not errs, "\n".join(errs)


async def test_deletes_template():
    s, c = new_secret("test-secret"), new_configmap("test-config")
    t = new_template("test", s, c, status={
        "syncedSecrets": ["test-secret"], "syncedConfigurations": ["test-config"], "syncedToClusters": ["shard0"],
        "conditions": [cond(True, 'Algorithm "test" ready')]})
    t_shard = new_template("test", s, c, on_shard=True)
    s_shard = new_secret("test-secret", t_shard)
    c_shard = new_configmap("test-config", t_shard)
    f = Fixture(ClusterFixture(template_list=[t], secret_list=[s], configmap_list=[c], existing_core=[s, c],
                               existing_nexus=[t]),
                ClusterFixture(template_list=[t_shard], secret_list=[s_shard], configmap_list=[c_shard],
                               existing_core=[s_shard, c_shard], existing_nexus=[t_shard]))
    f.expect_shard("delete", t_shard, R.TEMPLATES)
    errs = await f.run_object_handler([t])
    assert not errs, "\n".join(errs)


async def test_creates_workgroup():
    w = new_workgroup("test-workgroup", False, "shard0")
    f = Fixture(ClusterFixture(workgroup_list=[w], existing_nexus=[w]))
    f.expect_controller_status(expected_workgroup(w, [cond(False, 'Workgroup "test-workgroup" initializing')]),
                               R.WORKGROUPS)
    f.expect_controller_status(expected_workgroup(w, [cond(True, 'Workgroup "test-workgroup" ready')]), R.WORKGROUPS)
    f.expect_shard("create", expected_shard_workgroup(w, ""))
    errs = await f.run(workgroups=[(NS, "test-workgroup")])
    assert not errs, "\n".join(errs)


async def test_updates_workgroup():
    w = new_workgroup("test-workgroup", False, "shard0")
    w_shard = new_workgroup("test-workgroup", True, "shard0")
    w_upd = deep_copy(w)
    w_upd["spec"]["tolerations"] = [{"key": "key", "operator": "Exists"}]
    w_shard_upd = deep_copy(w_shard)
    w_shard_upd["spec"]["tolerations"] = w_upd["spec"]["tolerations"]
    f = Fixture(ClusterFixture(workgroup_list=[w_upd], existing_nexus=[w_upd]),
                ClusterFixture(workgroup_list=[w_shard], existing_nexus=[w_shard]))
    f.expect_controller_status(expected_workgroup(w_upd, [cond(False, 'Workgroup "test-workgroup" initializing')]),
                               R.WORKGROUPS)
    f.expect_controller_status(expected_workgroup(w_upd, [cond(True, 'Workgroup "test-workgroup" ready')]),
                               R.WORKGROUPS)
    f.expect_shard("update", expected_shard_workgroup(w_shard_upd, "test-workgroup"))
    errs = await f.run(workgroups=[(NS, "test-workgroup")])
    assert not errs, "\n".join(errs)
