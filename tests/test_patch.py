"""The fake apiserver's patch semantics (ncc/api/patch.py): RFC 7386 merge patch, RFC 6902 JSON patch, the
strategic-merge treatment of ownerReferences and the single-manager server-side-apply approximation."""
import pytest

from ncc.api.patch import apply_patch, json_patch, merge_patch, strategic_merge_patch


@pytest.mark.parametrize("target,patch,want", [  # RFC 7386 appendix A
    ({"a": "b"}, {"a": "c"}, {"a": "c"}),
    ({"a": "b"}, {"b": "c"}, {"a": "b", "b": "c"}),
    ({"a": "b"}, {"a": None}, {}),
    ({"a": "b", "b": "c"}, {"a": None}, {"b": "c"}),
    ({"a": ["b"]}, {"a": "c"}, {"a": "c"}),
    ({"a": "c"}, {"a": ["b"]}, {"a": ["b"]}),
    ({"a": {"b": "c"}}, {"a": {"b": "d", "c": None}}, {"a": {"b": "d"}}),
    ({"a": [{"b": "c"}]}, {"a": [1]}, {"a": [1]}),
    (["a", "b"], ["c", "d"], ["c", "d"]),
    ({"a": "b"}, ["c"], ["c"]),
    ({"a": "foo"}, None, None),
    ({"a": "foo"}, "bar", "bar"),
    ({"e": None}, {"a": 1}, {"e": None, "a": 1}),
    ([1, 2], {"a": "b", "c": None}, {"a": "b"}),
    ({}, {"a": {"bb": {"ccc": None}}}, {"a": {"bb": {}}}),
])
def test_merge_patch_rfc7386(target, patch, want):
    assert merge_patch(target, patch) == want


def test_json_patch_rfc6902_operations():
    doc = {"foo": ["bar", "baz"], "biscuits": [{"name": "Digestive"}, {"name": "Choco Leibniz"}], "a/b": 1, "m~n": 2}
    out = json_patch(doc, [
        {"op": "add", "path": "/foo/1", "value": "qux"},
        {"op": "add", "path": "/foo/-", "value": "end"},
        {"op": "replace", "path": "/foo/0", "value": "BAR"},
        {"op": "remove", "path": "/biscuits/0"},
        {"op": "test", "path": "/a~1b", "value": 1},
        {"op": "copy", "from": "/m~0n", "path": "/copied"},
        {"op": "move", "from": "/biscuits/0", "path": "/moved"},
        {"op": "add", "path": "/new", "value": {"x": [1]}},
        {"op": "remove", "path": "/new/x"},
    ])
    assert out == {"foo": ["BAR", "qux", "baz", "end"], "biscuits": [], "a/b": 1, "m~n": 2, "copied": 2,
                   "moved": {"name": "Choco Leibniz"}, "new": {}}
    assert doc["foo"] == ["bar", "baz"]  # the input is not modified
    assert json_patch(doc, [{"op": "replace", "path": "", "value": [1]}]) == [1]


@pytest.mark.parametrize("ops,err", [
    ([{"op": "test", "path": "/a", "value": 2}], ValueError),
    ([{"op": "replace", "path": "/missing", "value": 1}], KeyError),
    ([{"op": "remove", "path": ""}], ValueError),
    ([{"op": "add", "path": "no-slash", "value": 1}], ValueError),
])
def test_json_patch_errors(ops, err):
    with pytest.raises(err):
        json_patch({"a": 1}, ops)


def test_strategic_merge_patch_merges_owner_references_by_uid():
    live = {"metadata": {"name": "s", "ownerReferences": [{"uid": "1", "name": "a"}, {"uid": "2", "name": "b"}]},
            "data": {"k": "v"}}
    out = strategic_merge_patch(live, {"metadata": {"ownerReferences": [{"uid": "2", "name": "B"},
                                                                        {"uid": "3", "name": "c"}]},
                                       "data": {"k": None, "n": "w"}})
    assert [(r["uid"], r["name"]) for r in out["metadata"]["ownerReferences"]] == [("1", "a"), ("2", "B"), ("3", "c")]
    assert out["data"] == {"n": "w"} and out["metadata"]["name"] == "s"
    assert strategic_merge_patch(live, {"data": {"x": "y"}})["metadata"]["ownerReferences"] == \
        live["metadata"]["ownerReferences"]


def test_apply_patch_single_manager():
    applied = {"apiVersion": "v1", "kind": "Secret",
               "metadata": {"labels": {"app": "x"}, "annotations": {"a": "1"}, "ownerReferences": [{"uid": "u2"}]},
               "data": {"k": "bmV3"}}
    assert apply_patch(None, applied) == applied
    live = {"apiVersion": "v1", "kind": "Secret",
            "metadata": {"name": "s", "labels": {"keep": "y"}, "ownerReferences": [{"uid": "u1"}, {"uid": "u2"}]},
            "data": {"k": "b2xk", "other": "eA=="}, "type": "Opaque"}
    out = apply_patch(live, applied)
    assert out["metadata"]["labels"] == {"keep": "y", "app": "x"} and out["metadata"]["annotations"] == {"a": "1"}
    assert [r["uid"] for r in out["metadata"]["ownerReferences"]] == ["u1", "u2"]
    assert out["data"] == {"k": "bmV3"} and out["type"] == "Opaque" and out["metadata"]["name"] == "s"


def test_apply_removes_fields_its_applier_stopped_applying():
    """The fake apiserver's apply: a top-level field the applier set before and omits now is removed (real
    SSA does this from managedFields); fields set by a PUT, and re-created objects, start from scratch."""
    from ncc.api import resources as R
    from ncc.fakeapi.storage import ClusterState
    from ncc.kube.client import PATCH_APPLY

    st = ClusterState("shard")
    body = {"apiVersion": "v1", "kind": "ConfigMap", "metadata": {"name": "c", "namespace": "ns"},
            "data": {"a": "1"}, "binaryData": {"b": "AAE="}}
    st.patch(R.CONFIGMAPS, "ns", "c", body, PATCH_APPLY)
    slim = {k: v for k, v in body.items() if k != "binaryData"}
    out = st.patch(R.CONFIGMAPS, "ns", "c", slim, PATCH_APPLY)
    assert "binaryData" not in out and out["data"] == {"a": "1"}
    cur = st.get(R.CONFIGMAPS, "ns", "c")
    cur["binaryData"] = {"x": "AA=="}  # set by an update, not by the applier: an apply leaves it alone
    st.update(R.CONFIGMAPS, "ns", cur)
    assert st.patch(R.CONFIGMAPS, "ns", "c", slim, PATCH_APPLY)["binaryData"] == {"x": "AA=="}
    st.delete(R.CONFIGMAPS, "ns", "c")
    assert st._applied == {}
