"""Structural fingerprints: equal JSON ⇔ equal digest (native C++ walker and Python fallback)."""
import json

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from ncc import native
from ncc.api import fingerprint as F

NATIVE = native.load()
IMPLS = [F._py_fingerprint] + ([NATIVE.fingerprint] if NATIVE is not None else [])

json_values = st.recursive(
    st.none() | st.booleans() | st.integers(min_value=-2**70, max_value=2**70)
    | st.floats(allow_nan=False, allow_infinity=False) | st.text(max_size=20),
    lambda children: st.lists(children, max_size=5) | st.dictionaries(st.text(max_size=8), children, max_size=5),
    max_leaves=30)


@pytest.mark.parametrize("fp", IMPLS)
def test_key_order_does_not_matter(fp):
    a = {"spec": {"x": 1, "y": [1, 2, {"b": None, "a": "s"}]}, "z": True}
    b = {"z": True, "spec": {"y": [1, 2, {"a": "s", "b": None}], "x": 1}}
    assert fp(a) == fp(b)


@pytest.mark.parametrize("fp", IMPLS)
def test_types_and_order_are_distinguished(fp):
    distinct = [None, 0, 1, 1.5, "1", True, False, [], {}, [1, 2], [2, 1], {"a": 1}, {"a": "1"}, {"b": 1},
                [[]], [{}], "", "aé"]
    digests = [fp(v) for v in distinct]
    assert len(set(digests)) == len(distinct)


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
@settings(max_examples=400, deadline=None)
@given(json_values, json_values)
def test_native_equality_matches_json_equality(a, b):
    """Digest equality must agree with equality of the canonical JSON form (-0.0 folds to 0.0, as in Go ==)."""
    def norm(v):
        if isinstance(v, float) and v == 0.0:
            return 0.0
        if isinstance(v, list):
            return [norm(x) for x in v]
        if isinstance(v, dict):
            return {k: norm(x) for k, x in v.items()}
        return v
    ca = json.dumps(norm(a), sort_keys=True)
    cb = json.dumps(norm(b), sort_keys=True)
    assert (NATIVE.fingerprint(a) == NATIVE.fingerprint(b)) == (ca == cb)


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
def test_roundtrip_through_json_is_stable():
    from ncc.testing.workload import make_template
    t = make_template(7, "nexus", secrets=["s"], configmaps=["c"])
    assert NATIVE.fingerprint(t["spec"]) == NATIVE.fingerprint(json.loads(json.dumps(t["spec"])))
    assert NATIVE.fingerprint_many([t["spec"], None]) == [NATIVE.fingerprint(t["spec"]), NATIVE.fingerprint(None)]


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
def test_rejects_non_string_keys_and_deep_nesting():
    with pytest.raises(TypeError):
        NATIVE.fingerprint({1: "x"})
    deep = []
    cur = deep
    for _ in range(600):
        nxt = []
        cur.append(nxt)
        cur = nxt
    with pytest.raises(ValueError):
        NATIVE.fingerprint(deep)


def test_native_json_encoder_roundtrips():
    """ncc._native.dumps must decode to exactly what json.dumps does (UTF-8 instead of \\u escapes)."""
    import json
    from ncc.api.jsonenc import dumps_bytes
    from ncc.testing.workload import make_secret, make_template
    cases = [make_secret("s", "ns", payload=700, version=9), make_template(3, "ns", version="v9"),
             {"a": [1, -2, 2.5, -0.0, 1e300, 1.0, True, False, None], "s": "é☃ \n\t\"\\ \x01 \x1f /",
              "nested": {"x": {"y": [[], {}]}}, "big": 2 ** 80, "neg": -(2 ** 70)},
             [], {}, "plain", 7, None]
    for o in cases:
        assert json.loads(dumps_bytes(o)) == json.loads(json.dumps(o))
    assert dumps_bytes({1: "int key"}) == b'{"1":"int key"}'  # stdlib fallback semantics for odd keys


# ----------------------------------------------------------------------------- native JSON decoding
def _same(a, b) -> bool:
    """Equal values and equal types (1 vs 1.0 and -0.0 vs 0.0 count as different)."""
    if type(a) is not type(b):
        return False
    if isinstance(a, float):
        return str(a) == str(b)  # also tells -0.0 from 0.0, and nan == nan
    if isinstance(a, list):
        return len(a) == len(b) and all(_same(x, y) for x, y in zip(a, b))
    if isinstance(a, dict):
        return list(a) == list(b) and all(_same(a[k], b[k]) for k in a)
    return a == b


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
@settings(max_examples=400, deadline=None)
@given(json_values, st.booleans())
def test_native_loads_matches_stdlib(v, ascii_only):
    """`_native.loads` decodes what json.dumps writes (escaped or raw UTF-8) to exactly json.loads' value."""
    text = json.dumps(v, ensure_ascii=ascii_only)
    assert _same(NATIVE.loads(text.encode("utf-8", "surrogatepass")), json.loads(text))


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
@settings(max_examples=400, deadline=None)
@given(st.binary(max_size=64))
def test_native_loads_on_arbitrary_bytes(raw):
    """Malformed input gives None (the caller falls back to the stdlib); accepted input decodes as json does."""
    v = NATIVE.loads(raw)
    if v is None:
        return
    assert _same(v, json.loads(raw.decode("utf-8", "surrogatepass")))


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
def test_native_loads_edge_cases():
    from ncc.api.jsonenc import loads_fast
    for text in ['"\\ud83d\\ude00 \\u00e9 \\ud800 x"', "[1e400, -1e400, -0.0, 0, -0, 123456789012345678901234]",
                 '{"a": {"a": {"a": []}}, "b": "\\"\\\\\\/\\b\\f\\n\\r\\t"}', " [ ] ", "\"\"", "NaN"]:
        assert _same(loads_fast(text.encode("utf-8", "surrogatepass")), json.loads(text))
    for bad in [b"[1,]", b"{\"a\" 1}", b"01", b"[1] x", b"\"\x01\"", b"tru", b"-", b"1.", b"{\"a\":1,}"]:
        assert NATIVE.loads(bad) is None


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
def test_template_event_slim_keeps_what_the_coordinator_reads():
    """The coordinator's slim templates: metadata (without managedFields) and status decoded, the spec reduced
    to its Secret/ConfigMap references and a digest of the raw spec (same spec <=> same digest)."""
    from ncc.api.refs import dependent_names, same_references
    from ncc.testing.workload import make_template
    t = make_template(4, "nexus", secrets=["s1", "s2"], configmaps=["c1"], version="v1")
    t["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"].insert(1, {"prefix": "X_", "secretRef": None})
    t["metadata"].update(uid="u-4", resourceVersion="77", generation=3,
                         managedFields=[{"manager": "kubectl", "fieldsV1": {"f:spec": {}}}])
    t["status"] = {"conditions": [{"type": "Ready", "status": "True", "message": "Algorithm \"é\" ready"}],
                   "syncedSecrets": ["s1", "s2"]}
    line = json.dumps({"type": "MODIFIED", "object": t}).encode()
    typ, slim = NATIVE.template_event_slim(line)
    assert typ == "MODIFIED" and slim["kind"] == t["kind"] and slim["apiVersion"] == t["apiVersion"]
    assert slim["status"] == t["status"]
    assert slim["metadata"] == {k: v for k, v in t["metadata"].items() if k != "managedFields"}
    assert dependent_names(slim) == dependent_names(t) == (["s1", "s2"], ["c1"])
    assert same_references(slim, t)
    again = NATIVE.template_event_slim(json.dumps({"object": t, "type": "MODIFIED"}).encode())[1]
    assert again["spec"] == slim["spec"]
    t["spec"]["container"]["versionTag"] = "v2"
    changed = NATIVE.template_event_slim(json.dumps({"type": "MODIFIED", "object": t}).encode())[1]
    assert changed["spec"] != slim["spec"] and dependent_names(changed) == dependent_names(slim)
    no_env = dict(t, spec={"container": {}})
    assert dependent_names(NATIVE.template_event_slim(json.dumps({"type": "ADDED", "object": no_env}).encode())[1]) \
        == ([], [])
    for bad in [b"", b"{}", b'{"type": "ADDED"}', b'{"type": "ADDED", "object": {"spec": [}}', line[:-1]]:
        assert NATIVE.template_event_slim(bad) is None


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
def test_template_event_slim_reuses_unchanged_parts_of_the_cached_version():
    """With the store's items, an unchanged status and an unchanged reference list are the cached version's
    objects (not decoded again); a changed one is decoded; the result equals the uncached decode either way."""
    from ncc.testing.workload import make_template
    t = make_template(5, "nexus", secrets=["s1"], configmaps=["c1"], version="v1")
    t["metadata"].update(uid="u-5", resourceVersion="10", generation=1)
    t["status"] = {"conditions": [{"type": "Ready", "status": "True"}], "syncedSecrets": ["s1"]}
    line = lambda: json.dumps({"type": "MODIFIED", "object": t}).encode()  # noqa: E731
    first = NATIVE.template_event_slim(line())[1]
    items = {("nexus", t["metadata"]["name"]): first}
    t["metadata"]["resourceVersion"] = "11"
    t["spec"]["container"]["versionTag"] = "v2"
    second = NATIVE.template_event_slim(line(), items, "")[1]
    assert second == NATIVE.template_event_slim(line())[1]
    assert second["status"] is first["status"]
    env = "runtimeEnvironment", "mappedEnvironmentVariables"
    assert second["spec"][env[0]][env[1]] is first["spec"][env[0]][env[1]]
    assert second["spec"]["_fp"] != first["spec"]["_fp"]
    t["status"]["syncedSecrets"] = []
    t["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"].append({"prefix": "Y_"})
    third = NATIVE.template_event_slim(line(), {("nexus", t["metadata"]["name"]): second}, "")[1]
    assert third == NATIVE.template_event_slim(line())[1]
    assert third["status"] is not second["status"] and third["status"]["syncedSecrets"] == []
    assert third["spec"]["_rfp"] != second["spec"]["_rfp"]
    # the namespace defaults when the object carries none
    del t["metadata"]["namespace"]
    fourth = NATIVE.template_event_slim(line(), {("nexus", t["metadata"]["name"]): third}, "nexus")[1]
    assert fourth["status"] is third["status"]
