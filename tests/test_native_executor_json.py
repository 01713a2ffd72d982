"""The native executor's JSON layer (native/executor/json.hpp), driven through `ncc-executor --json-selftest`:
the streaming fingerprint of raw payload text equals the fingerprint of its parsed DOM (the executor compares
controller-side payloads it never decodes against shard copies it did decode), and an object split into
metadata + raw payloads renders back to the same JSON value."""
import json
import os
import subprocess

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "ncc", "bin", "ncc-executor")

pytestmark = pytest.mark.skipif(not os.path.exists(EXE), reason="native executor not built")

scalars = (st.none() | st.booleans() | st.integers(min_value=-2**60, max_value=2**60)
           | st.floats(allow_nan=False, allow_infinity=False, width=32) | st.text(max_size=12))
values = st.recursive(scalars, lambda c: st.lists(c, max_size=4) | st.dictionaries(st.text(max_size=6), c, max_size=4),
                      max_leaves=25)


def run(texts):
    out = subprocess.run([EXE, "--json-selftest"], input="\n".join(texts) + "\n", capture_output=True, text=True,
                         timeout=60, check=True).stdout.split("\n")[:-1]  # (not splitlines: U+0085 etc. are data)
    assert len(out) == len(texts)
    return [line.split(" ", 2) for line in out]


@settings(max_examples=60, deadline=None)
@given(st.lists(values, min_size=1, max_size=20), st.booleans())
def test_streaming_fingerprint_equals_dom_fingerprint(vs, ascii_only):
    texts = [json.dumps(v, ensure_ascii=ascii_only) for v in vs]
    for text, (a, b, _) in zip(texts, run(texts)):
        assert a == b, text


@settings(max_examples=60, deadline=None)
@given(st.lists(st.fixed_dictionaries({"metadata": st.dictionaries(st.text(max_size=5), scalars, max_size=3)},
                                      optional={"spec": values, "data": values, "kind": st.text(max_size=4)}),
                min_size=1, max_size=20))
def test_split_render_round_trips(objs):
    texts = [json.dumps(o) for o in objs]
    for o, (_, _, render) in zip(objs, run(texts)):
        assert json.loads(render) == o


def test_fingerprint_text_semantics():
    texts = ['{"a": 1, "b": [1, 2]}', '{"b":[1,2],"a":1.0}', '{"a":"\\u00e9\\ud83d\\ude00"}', '{"a":"é😀"}',
             "[]", "{}", "null", "[1,[2,[3]]]", '"\\/"']
    fps = [a for a, b, _ in run(texts) if a == b]
    assert len(fps) == len(texts)
    assert fps[0] == fps[1]  # member order and 1 == 1.0 do not matter
    assert fps[2] == fps[3]  # escapes decode to the same string
    assert len({fps[4], fps[5], fps[6]}) == 3
