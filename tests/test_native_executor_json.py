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


names = st.text(alphabet=st.characters(min_codepoint=32, max_codepoint=0x2FF), max_size=8)
owner_ref = st.fixed_dictionaries({"apiVersion": st.just("science.sneaksanddata.com/v1"),
                                   "kind": st.sampled_from(["NexusAlgorithmTemplate", "Other"]),
                                   "name": names, "uid": names})
shard_objs = st.fixed_dictionaries(
    {"metadata": st.fixed_dictionaries(
        {"name": names, "resourceVersion": st.integers(0, 10**9).map(str)},
        optional={"namespace": names, "uid": names, "ownerReferences": st.none() | st.lists(owner_ref, max_size=3),
                  "labels": st.none() | st.dictionaries(
                      st.sampled_from(["science.sneaksanddata.com/controller-app",
                                       "science.sneaksanddata.com/configuration-owner", "x"]), names, max_size=3),
                  "annotations": st.dictionaries(names, names, max_size=2)})},
    optional={"spec": values, "status": values, "data": st.none() | st.dictionaries(names, names, max_size=3),
              "binaryData": st.none() | st.dictionaries(names, names, max_size=2), "type": st.none() | names,
              "apiVersion": st.just("v1"), "kind": st.sampled_from(["Secret", "ConfigMap", "NexusAlgorithmTemplate"])})


@settings(max_examples=80, deadline=None)
@given(st.lists(shard_objs, min_size=1, max_size=15), st.booleans())
def test_shard_object_scan_matches_the_dom_path(objs, ascii_only):
    """The executor reads write responses without a DOM (`shard_obj_scan`): for every object it accepts, the
    slim fields and fingerprints equal the DOM path's and the kept text is the same object without its
    payloads; anything it refuses (escaped strings) takes the DOM path."""
    texts = [json.dumps(o, ensure_ascii=ascii_only) for o in objs]
    out = subprocess.run([EXE, "--shardobj-selftest"], input="\n".join(texts) + "\n", capture_output=True,
                         text=True, timeout=60, check=True).stdout.split("\n")[:-1]
    assert len(out) == 2 * len(texts)
    for i, line in enumerate(out):
        fast, same, rest_fast, rest_slow = line.split("\t")
        if fast == "1":
            assert same == "1", (texts[i // 2], line)
            assert json.loads(rest_fast) == json.loads(rest_slow)



def test_plain_shard_object_takes_the_scan_path():
    obj = {"apiVersion": "v1", "kind": "Secret", "type": "Opaque", "data": {"k": "dg=="},
           "metadata": {"name": "s0", "namespace": "nexus", "uid": "u1", "resourceVersion": "42",
                        "labels": {"science.sneaksanddata.com/controller-app": "nexus-configuration-controller"},
                        "ownerReferences": [{"apiVersion": "science.sneaksanddata.com/v1",
                                             "kind": "NexusAlgorithmTemplate", "name": "t", "uid": "tu"}]}}
    out = subprocess.run([EXE, "--shardobj-selftest"], input=json.dumps(obj) + "\n", capture_output=True, text=True,
                         timeout=60, check=True).stdout.split("\n")[:-1]
    assert [line.split("\t")[:2] for line in out] == [["1", "1"], ["1", "1"]]


@settings(max_examples=80, deadline=None)
@given(st.lists(st.tuples(st.sampled_from(["ADDED", "MODIFIED", "DELETED"]), shard_objs,
                          st.none() | st.integers(0, 50),
                          st.lists(st.sampled_from(["s1", "s2"]), max_size=2),
                          st.lists(st.sampled_from(["c1"]), max_size=1)), min_size=1, max_size=15),
       st.booleans())
def test_relayed_line_scan_matches_the_dom_path(events, ascii_only):
    """The executor reads relayed controller-side watch lines without a DOM of their metadata (`ctl_scan`):
    every field of the resulting object — keys, resourceVersion, generation, label/annotation and payload
    fingerprints, raw payloads, references, owners — equals what the parser path builds."""
    texts = []
    for typ, obj, gen, secs, cms in events:
        obj = json.loads(json.dumps(obj))
        if gen is not None:
            obj["metadata"]["generation"] = gen
        if isinstance(obj.get("spec"), dict) or "spec" not in obj:
            obj["spec"] = {"runtimeEnvironment": {"mappedEnvironmentVariables": [
                {"secretRef": {"name": n}} for n in secs] + [{"configMapRef": {"name": n}} for n in cms]}}
        texts.append(json.dumps({"type": typ, "object": obj}, ensure_ascii=ascii_only))
    out = subprocess.run([EXE, "--shardobj-selftest"], input="\n".join(texts) + "\n", capture_output=True,
                         text=True, timeout=60, check=True).stdout.split("\n")[:-1]
    assert len(out) == 2 * len(texts)
    for i, line in enumerate(out):
        fast, same = line.split("\t")[:2]
        assert fast != "-1", (texts[i // 2], line)  # the scan never raises on a line the parser reads
        if fast == "1":
            assert same == "1", (texts[i // 2], line)


def test_plain_relayed_line_takes_the_scan_path():
    ev = {"type": "MODIFIED", "object": {
        "apiVersion": "science.sneaksanddata.com/v1", "kind": "NexusAlgorithmTemplate",
        "metadata": {"name": "t", "namespace": "nexus", "uid": "u", "resourceVersion": "7", "generation": 3,
                     "labels": {"a": "b"}},
        "spec": {"runtimeEnvironment": {"mappedEnvironmentVariables": [{"secretRef": {"name": "s"}}]}}}}
    out = subprocess.run([EXE, "--shardobj-selftest"], input=json.dumps(ev) + "\n", capture_output=True, text=True,
                         timeout=60, check=True).stdout.split("\n")[:-1]
    assert [line.split("\t")[:2] for line in out] == [["1", "1"], ["1", "1"]]


_json_leaf = st.none() | st.booleans() | st.integers() | st.text(alphabet=st.sampled_from(
    list('ab"\\{}[]:, é中') + ["\n"]), max_size=90)
_json_tree = st.recursive(_json_leaf, lambda kids: st.lists(kids, max_size=6) |
                          st.dictionaries(st.text(alphabet='ab"\\{[', max_size=8), kids, max_size=6), max_leaves=40)


@settings(max_examples=300, deadline=None)
@given(st.lists(st.tuples(_json_tree.filter(lambda v: isinstance(v, (list, dict))), st.booleans(),
                          st.sampled_from(["", ",\"x\":1}", "]]", " {\"a\":[1]}"])), min_size=1, max_size=20))
def test_container_skip_matches_a_json_decoder(cases):
    """skip_container_text (json.hpp: 64-byte blocks of quote/backslash/bracket bit masks, byte by byte
    where a block has a backslash) ends each container exactly where a JSON decoder does: strings full of
    brackets, quotes and backslashes, values straddling block edges, trailing text after the container."""
    lines, want = [], []
    for value, compact, tail in cases:
        text = json.dumps(value, ensure_ascii=False, separators=(",", ":") if compact else None)
        _, end = json.JSONDecoder().raw_decode(text + tail)
        lines.append(text + tail)
        want.append(len((text + tail)[:end].encode()))
    out = subprocess.run([EXE, "--skip-selftest"], input="\n".join(lines) + "\n", capture_output=True, text=True,
                         timeout=60, check=True).stdout.split()
    assert [int(x) for x in out] == want


def test_decode_bench_reads_both_paths():
    """`ncc-executor --decode-bench KIND` (the relayed-line decode microbenchmark) reports a time per line
    for the parser path and the scan path over the same lines."""
    ev = {"type": "ADDED", "object": {"metadata": {"name": "s", "namespace": "nexus", "resourceVersion": "1"},
                                      "data": {"k": "dg=="}}}
    out = subprocess.run([EXE, "--decode-bench", "2"], input=json.dumps(ev) + "\n", capture_output=True, text=True,
                         timeout=60, check=True).stdout
    d = json.loads(out)
    assert d["lines"] == 1 and d["parser_ns"] > 0 and d["scan_ns"] > 0


_mp_leaf = (st.none() | st.booleans() | st.integers(-(2 ** 63), 2 ** 63 - 1) |
            st.floats(allow_nan=False, allow_infinity=False, min_value=-1e38, max_value=1e38) |
            st.text(max_size=300) | st.binary(max_size=300))
_mp_tree = st.recursive(_mp_leaf, lambda kids: st.lists(kids, max_size=20) |
                        st.dictionaries(st.text(max_size=6), kids, max_size=20), max_leaves=60)


def _mp_expect(v):
    if isinstance(v, dict):
        return [[k, _mp_expect(x)] for k, x in v.items()]
    if isinstance(v, list):
        return [_mp_expect(x) for x in v]
    if isinstance(v, bytes):
        return {"bin": v.hex()}
    return v


def _mp_encodable(v):
    if isinstance(v, dict):
        return all(_mp_encodable(x) for x in v.values())
    if isinstance(v, list):
        return all(_mp_encodable(x) for x in v)
    return not isinstance(v, (float, bytes))


@settings(max_examples=150, deadline=None)
@given(st.lists(st.tuples(_mp_tree, st.booleans()), min_size=1, max_size=10))
def test_msgpack_decoder_and_encoder_against_msgpack(values):
    """The executor's msgpack layer (native/executor/msgpack.hpp, the socketpair protocol) against the Python
    msgpack package: every width of int/str/bin/array/map, single and double floats, and nesting decode to
    the same value; what the executor itself sends (no floats, no bin) re-encodes to bytes msgpack reads back
    as the same value."""
    import msgpack
    blobs = [msgpack.packb(v, use_bin_type=True, use_single_float=single) for v, single in values]
    blobs.append(b"\xc1")  # never used: an error, not a crash
    out = subprocess.run([EXE, "--msgpack-selftest"], input="\n".join(b.hex() for b in blobs) + "\n",
                         capture_output=True, text=True, timeout=60, check=True).stdout.split("\n")[:-1]
    assert len(out) == len(blobs) and out[-1] == "error"
    for (v, single), line in zip(values, out):
        rendered, re = line.split("\t")
        want = msgpack.unpackb(msgpack.packb(v, use_single_float=single), raw=False) if single else v
        assert json.loads(rendered) == _mp_expect(want)
        if _mp_encodable(v):
            assert msgpack.unpackb(bytes.fromhex(re), raw=False, strict_map_key=False) == v
        else:
            assert re == "-"
