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
