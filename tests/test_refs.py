"""Template reference helpers (`ncc/api/refs.py`).

`GetSecretNames()` / `GetConfigMapNames()` read
`spec.runtimeEnvironment.mappedEnvironmentVariables[*].{secretRef,configMapRef}.name` and skip entries
without that ref; the reference fixture builds zero-valued `EnvFromSource` entries when refs are nil
(controller_test.go:261-282).
"""
from ncc.api import constants as C
from ncc.api.refs import (configmap_names, dependent_names, is_owned_by_uid, same_references, secret_names,
                          template_owner_names, template_owner_ref)


def _template(env, name="algo", uid="u-1", rv="1"):
    return {"apiVersion": C.API_VERSION, "kind": C.TEMPLATE_KIND,
            "metadata": {"name": name, "namespace": "nexus", "uid": uid, "resourceVersion": rv},
            "spec": {"runtimeEnvironment": {"mappedEnvironmentVariables": env}}}


ENV = [
    {"secretRef": {"name": "s1"}},
    {"configMapRef": {"name": "c1"}},
    {},                                   # zero-valued EnvFromSource
    None,
    {"secretRef": {"name": "s2"}, "configMapRef": {"name": "c2"}},
    {"secretRef": {"name": "s1"}},        # duplicate reference
]


def test_names_skip_entries_without_ref_and_keep_order():
    t = _template(ENV)
    assert secret_names(t) == ["s1", "s2", "s1"]
    assert configmap_names(t) == ["c1", "c2"]
    assert secret_names(t, unique=True) == ["s1", "s2"]


def test_dependent_names_matches_the_two_walks():
    for env in (ENV, [], [None, {}], [{"configMapRef": {}}]):
        t = _template(env)
        assert dependent_names(t) == (secret_names(t), configmap_names(t))


def test_missing_spec_sections_yield_no_names():
    for t in ({}, {"spec": None}, {"spec": {"runtimeEnvironment": None}},
              {"spec": {"runtimeEnvironment": {"mappedEnvironmentVariables": None}}}):
        assert secret_names(t) == [] and configmap_names(t) == [] and dependent_names(t) == ([], [])


def test_same_references():
    old = _template(ENV, rv="1")
    assert same_references(old, _template([dict(e) if e else e for e in ENV], rv="2"))
    # Different entry shapes, same referenced names (an extra empty entry) → same references.
    assert same_references(old, _template(ENV + [{}], rv="2"))
    # A renamed, added or reordered reference is a change.
    assert not same_references(old, _template(ENV[:-1] + [{"secretRef": {"name": "s3"}}]))
    assert not same_references(old, _template(ENV + [{"configMapRef": {"name": "c3"}}]))
    assert not same_references(_template([{"secretRef": {"name": "a"}}, {"secretRef": {"name": "b"}}]),
                               _template([{"secretRef": {"name": "b"}}, {"secretRef": {"name": "a"}}]))


def test_owner_ref_and_ownership():
    t = _template(ENV)
    ref = template_owner_ref(t)
    assert ref == {"apiVersion": C.API_VERSION, "kind": C.TEMPLATE_KIND, "name": "algo", "uid": "u-1"}
    assert "controller" not in ref and "blockOwnerDeletion" not in ref
    dep = {"metadata": {"ownerReferences": [ref, {"kind": "Deployment", "name": "x", "uid": "u-9"}]}}
    assert is_owned_by_uid(dep, "u-1") and is_owned_by_uid(dep, "u-9")
    assert not is_owned_by_uid(dep, "u-2") and not is_owned_by_uid({"metadata": {}}, "u-1")
    assert template_owner_names(dep) == ["algo"]
