"""The coordinator's report table: the native ReportTable (native/ncc_native.cpp) against its Python twin
(ncc/controller/reports.py), driven in lock-step with arbitrary report streams, frames and shard-set
changes; plus the raw-frame path through ipc.Channel and Controller.on_executor_frame."""
import asyncio
import socket

import msgpack
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from ncc import native
from ncc.controller.ipc import Channel
from ncc.controller.reports import ReportTable

NATIVE = native.load()

SHARDS = ["s0", "s1", "s2"]
KEYS = ["NexusAlgorithmTemplate/ns/a", "NexusAlgorithmTemplate/ns/b", "NexusAlgorithmWorkgroup/ns/w"]

# typed failures (ncc/controller/failures.py): kept raw by the native table, decoded back by readiness()
failure = st.fixed_dictionaries({"c": st.sampled_from(["RogueResourceError", "Conflict", "TransportError"]),
                                 "k": st.sampled_from(["", "Secret", "NexusAlgorithmTemplate"]),
                                 "n": st.sampled_from(["", "s0"]), "h": st.integers(0, 600),
                                 "m": st.text(max_size=6)})
report = st.fixed_dictionaries({
    "t": st.just("report"), "k": st.sampled_from(KEYS), "u": st.sampled_from(["u1", "u2"]),
    "g": st.integers(0, 4), "r": st.dictionaries(st.sampled_from(SHARDS + ["gone"]),
                                                 st.one_of(st.none(), st.just(""), st.sampled_from(["boom", "409"]),
                                                           failure),
                                                 min_size=1, max_size=3),
    "w": st.booleans()})
other = st.one_of(
    st.fixed_dictionaries({"t": st.sampled_from(["ready", "synced"]), "i": st.integers(0, 1 << 40)}),
    st.fixed_dictionaries({"t": st.just("need"), "k": st.integers(0, 3), "n": st.text(max_size=8)}),
    st.fixed_dictionaries({"t": st.just("x"), "f": st.floats(allow_nan=False), "b": st.binary(max_size=4),
                           "l": st.lists(st.one_of(st.none(), st.booleans(), st.integers(-(1 << 63), (1 << 64) - 1)),
                                         max_size=3)}))
op = st.one_of(
    st.tuples(st.just("feed"), st.lists(st.one_of(report, report, other), min_size=1, max_size=5)),
    st.tuples(st.just("shards"), st.lists(st.sampled_from(SHARDS), unique=True, max_size=3)),
    st.tuples(st.just("drop"), st.lists(st.sampled_from(SHARDS), max_size=2)),
    st.tuples(st.just("pop"), st.sampled_from(KEYS)),
    st.tuples(st.just("part"), st.integers(1, 3).flatmap(lambda c: st.tuples(st.integers(0, c - 1), st.just(c)))))


def frame(msgs: list) -> tuple[bytes, bool]:
    if len(msgs) == 1:
        return msgpack.packb(msgs[0], use_bin_type=True), False
    return msgpack.packb(msgs, use_bin_type=True), True


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
@settings(max_examples=300, deadline=None)
@given(st.lists(op, max_size=25))
def test_native_report_table_matches_python(ops):
    py, nat = ReportTable(), NATIVE.ReportTable()
    for t in (py, nat):
        t.set_shards(SHARDS[:2])
    for kind, arg in ops:
        if kind == "feed":
            body, batch = frame(arg)
            assert nat.feed(body, batch) == py.feed(body, batch)
            fn, fp = nat.take_forwards(), py.take_forwards()
            assert {p: [msgpack.unpackb(m) for m in ms] for p, ms in fn.items()} == \
                {p: [msgpack.unpackb(m) for m in ms] for p, ms in fp.items()}
        elif kind == "part":
            py.set_partition(*arg), nat.set_partition(*arg)
        elif kind == "shards":
            py.set_shards(arg), nat.set_shards(arg)
            assert nat.shards() == py.shards() == arg
        elif kind == "drop":
            py.drop_shards(arg), nat.drop_shards(arg)
        else:
            py.pop(arg), nat.pop(arg)
        assert len(nat) == len(py)
        for k in KEYS:
            for u in ("u1", "u2"):
                for g in range(5):
                    assert nat.readiness(k, u, g) == py.readiness(k, u, g)
                    assert nat.ready_ok(k, u, g) == py.ready_ok(k, u, g)


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
@settings(max_examples=300, deadline=None)
@given(st.binary(max_size=48), st.booleans())
def test_native_report_table_rejects_malformed_frames(raw, batch):
    """Arbitrary bytes either fold like the Python twin or raise (ValueError for a malformed frame, what
    msgpack raises for undecodable content: bad UTF-8, an unhashable map key); never crash."""
    nat, py = NATIVE.ReportTable(), ReportTable()
    nat.set_shards(SHARDS), py.set_shards(SHARDS)
    try:
        got = nat.feed(raw, batch)
    except (ValueError, UnicodeDecodeError, TypeError):
        return
    try:
        want = py.feed(raw, batch)
    except Exception:  # noqa: BLE001 — msgpack is laxer about some inputs the native table refuses
        return
    if got[4] or want[4]:  # only well-formed reports are compared
        assert got[:3] == want[:3]


def framed(frames: list) -> bytes:
    out = b""
    for msgs in frames:
        body, batch = frame(msgs)
        out += (len(body) | (0x80000000 if batch else 0)).to_bytes(4, "big")
        out += body
    return out


@pytest.mark.skipif(NATIVE is None, reason="native extension not built")
@settings(max_examples=200, deadline=None)
@given(st.lists(st.lists(st.one_of(report, other), min_size=1, max_size=4), min_size=1, max_size=6),
       st.lists(st.integers(0, 400), max_size=5))
def test_native_feed_stream_matches_python_at_any_split(frames, cuts):
    """A frame stream cut into arbitrary reads folds the same natively and in Python, and as a whole."""
    data = framed(frames)
    cuts = sorted({min(c, len(data)) for c in cuts} | {len(data)})
    results = []
    for t in (NATIVE.ReportTable(), ReportTable()):
        t.set_shards(SHARDS[:2])
        buf, pos, got, prev = bytearray(), 0, [[], [], [], [], 0, 0], 0
        for c in cuts:  # what Channel.recv_folded does with each read
            buf += data[prev:c]
            prev = c
            r = t.feed_stream(buf, pos)
            for i in range(4):
                got[i] += r[i]
            got[4] += r[4]
            got[5] += r[5]
            pos = r[6]
        assert pos == len(buf)
        results.append(got)
    assert results[0] == results[1]
    whole = NATIVE.ReportTable()
    whole.set_shards(SHARDS[:2])
    r = whole.feed_stream(data, 0)
    assert list(r[:4]) == results[0][:4] and r[4:6] == tuple(results[0][4:6]) and r[6] == len(data)


def test_feed_stream_bounds():
    """A frame header past the 64 MiB cap is an error, a partial header or body is left for the next read,
    and `start` past the end is refused."""
    for t in ([NATIVE.ReportTable()] if NATIVE is not None else []) + [ReportTable()]:
        with pytest.raises(ValueError):
            t.feed_stream(b"\x7f\xff\xff\xff" + b"x" * 8, 0)
        body = msgpack.packb({"t": "ready", "i": 1})
        data = len(body).to_bytes(4, "big") + body
        assert t.feed_stream(data[:3], 0)[6] == 0 and t.feed_stream(data[:-1], 0)[6] == 0
        assert t.feed_stream(data, 0)[3] == [{"t": "ready", "i": 1}] and t.feed_stream(data, 0)[6] == len(data)
        assert t.feed_stream(b"pad" + data, 3)[6] == 3 + len(data)
    if NATIVE is not None:
        with pytest.raises(ValueError):
            NATIVE.ReportTable().feed_stream(b"abc", 4)


def test_report_table_completion_and_readiness():
    t = (NATIVE.ReportTable if NATIVE is not None else ReportTable)()
    t.set_shards(["a", "b"])
    k = "NexusAlgorithmTemplate/ns/x"
    assert t.feed(*frame([{"t": "report", "k": k, "u": "u", "g": 2, "r": {"a": None}, "w": True}])) == \
        ([], [k], [], [], 1, 1)
    assert t.readiness(k, "u", 2) is None
    got = t.feed(*frame([{"t": "report", "k": k, "u": "u", "g": 2, "r": {"b": "boom"}, "w": False},
                         {"t": "need", "k": 1, "n": "ns/s"}]))
    assert got == ([k], [], ["b"], [{"t": "need", "k": 1, "n": "ns/s"}], 1, 0)
    assert t.readiness(k, "u", 2) == {"a": None, "b": "boom"} and t.ready_ok(k, "u", 2) is False
    assert t.readiness(k, "u", 3) is None and t.readiness(k, "other", 2) is None and t.ready_ok(k, "u", 3) is None
    # a repeat of a complete set with nothing new is not a completion; a changed result or a write is
    rep = {"t": "report", "k": k, "u": "u", "g": 2, "r": {"a": None}, "w": False}
    assert t.feed(*frame([rep])) == ([], [], [], [], 1, 0)
    assert t.feed(*frame([dict(rep, w=True)])) == ([k], [k], [], [], 1, 0)
    assert t.feed(*frame([dict(rep, r={"b": None})])) == ([k], [], [], [], 1, 0)
    assert t.readiness(k, "u", 2) == {"a": None, "b": None} and t.ready_ok(k, "u", 2) is True
    t.set_shards(["a", "b", "c"])  # a shard added: not complete until it reports
    assert t.readiness(k, "u", 2) is None
    t.drop_shards(["c"])
    t.set_shards(["a", "b"])
    assert t.readiness(k, "u", 2) == {"a": None, "b": None}
    t.pop(k)
    assert t.readiness(k, "u", 2) is None and len(t) == 0


async def test_channel_raw_frames_fold_through_the_controller_path():
    """Frames written by Channel.send (single and coalesced batches) arrive undecoded via recv_raw and fold
    exactly as their decoded messages would."""
    a, b = socket.socketpair()
    ra, wa = await asyncio.open_connection(sock=a)
    rb, wb = await asyncio.open_connection(sock=b)
    tx, rx = Channel(ra, wa), Channel(rb, wb)
    t = (NATIVE.ReportTable if NATIVE is not None else ReportTable)()
    t.set_shards(["s0"])
    tx.send({"t": "report", "k": "K/ns/a", "u": "u", "g": 1, "r": {"s0": None}, "w": True})
    await tx.drain()
    body, batch = await rx.recv_raw()
    assert not batch and t.feed(body, batch)[:2] == (["K/ns/a"], ["K/ns/a"])
    tx.send({"t": "ready", "i": 0})
    tx.send({"t": "report", "k": "K/ns/b", "u": "u", "g": 1, "r": {"s0": "boom"}, "w": False})
    await tx.drain()
    body, batch = await rx.recv_raw()
    assert batch and t.feed(body, batch) == (["K/ns/b"], [], ["s0"], [{"t": "ready", "i": 0}], 1, 0)
    # the folding path: frames cut across reads are folded once complete; other messages come back decoded
    t2 = (NATIVE.ReportTable if NATIVE is not None else ReportTable)()
    t2.set_shards(["s0"])
    seen = []

    def fold(buf, start):
        r = t2.feed_stream(buf, start)
        seen.extend(r[0])
        return r[3], r[6]
    data = framed([[{"t": "report", "k": "K/ns/c", "u": "u", "g": 1, "r": {"s0": None}, "w": False}],
                   [{"t": "synced", "i": 3}]])
    wa.write(data[:7])
    await wa.drain()
    assert await rx.recv_folded(fold) == [] and seen == []
    wa.write(data[7:])
    await wa.drain()
    got = []
    while not got:
        got = await rx.recv_folded(fold)
    assert got == [{"t": "synced", "i": 3}] and seen == ["K/ns/c"]
    tx.close()
    assert await rx.recv_folded(fold) is None
    rx.close()


# ------------------------------------------------------------------ the coordinator's template on_update
_val = st.one_of(st.none(), st.sampled_from(["1", "2", "3"]))
_meta = st.fixed_dictionaries({}, optional={
    "namespace": st.sampled_from(["ns", "", None]), "name": st.sampled_from(["a", "b"]),
    "resourceVersion": _val, "uid": st.sampled_from(["u1", "u2", "", None]),
    "generation": st.one_of(st.none(), st.integers(0, 3)),
    "labels": st.one_of(st.none(), st.just({}), st.just({"x": "1"})),
    "annotations": st.one_of(st.none(), st.just({"y": "1"}))})
_env = st.sampled_from([[], [{"name": "E", "valueFrom": {"secretKeyRef": {"name": "s0", "key": "k"}}}],
                        [{"name": "E", "valueFrom": {"configMapKeyRef": {"name": "c0", "key": "k"}}}]])
_spec = st.one_of(st.none(), st.just({}),
                  st.fixed_dictionaries({"runtimeEnvironment": st.fixed_dictionaries({"mappedEnvironmentVariables": _env}),
                                         "container": st.sampled_from([{"image": "a"}, {"image": "b"}])},
                                        optional={"_rfp": st.sampled_from([1, 2])}))
_status = st.one_of(st.none(), st.just({}), st.just({"conditions": []}),
                    st.just({"conditions": [{"type": "Ready", "status": "True"}]}))
_template = st.fixed_dictionaries({}, optional={"metadata": _meta, "spec": _spec, "status": _status})


@pytest.mark.skipif(NATIVE is None or not hasattr(NATIVE.ReportTable(), "template_update"),
                    reason="native extension not built")
@settings(max_examples=600, deadline=None)
@given(old=_template, new=_template, adopted=st.dictionaries(st.sampled_from(["template/ns/a", "template//a",
                                                                              "template/ns/b"]), _val, max_size=3),
       reports=st.lists(st.tuples(st.sampled_from(["template/ns/a", "template//a"]), st.sampled_from(["u1", "u2"]),
                                  st.integers(0, 3)), max_size=3),
       gf=st.booleans())
def test_native_template_update_matches_the_python_handler(old, new, adopted, reports, gf):
    """`ReportTable.template_update` (the coordinator's template on_update in one native call) decides as
    `Controller._on_crd_update` does — enqueue, skip the early pass, or nothing — and leaves the adoption cache
    the same; inputs it does not handle raise TypeError (the handler then runs in Python)."""
    from types import SimpleNamespace

    from ncc.api.refs import same_references
    from ncc.controller.controller import Controller
    table = NATIVE.ReportTable()
    table.set_shards(["s0", "s1"])
    for key, uid, gen in reports:
        for sh in ("s0", "s1"):
            table.feed(*frame([{"t": "report", "k": key, "u": uid, "g": gen, "r": {sh: None}, "w": False}]))
    enq = []
    stub = SimpleNamespace(options=SimpleNamespace(adoption_cache=True, generation_filter=gf), role="coordinator",
                           _adopted=dict(adopted), stats={"early_passes_skipped": 0}, reports=table,
                           _enqueue_key=enq.append)
    stub.shard_ready_ok = lambda key, obj: Controller.shard_ready_ok(stub, key, obj)
    try:
        Controller._on_crd_update(stub, old, new, "template")
        want = ("ok", enq[0] if enq else None, stub.stats["early_passes_skipped"], stub._adopted)
    except (TypeError, AttributeError) as e:
        want = ("error", type(e).__name__)
    nat_adopted = dict(adopted)
    try:
        r = table.template_update(old, new, nat_adopted, gf, same_references)
        got = ("ok", r if isinstance(r, str) else None, 1 if r is False else 0, nat_adopted)
    except TypeError:
        got = None  # the Python handler decides
    if got is not None:
        assert got == want, (old, new, adopted)


@pytest.mark.skipif(NATIVE is None or not hasattr(NATIVE, "template_index_same"), reason="native extension not built")
@settings(max_examples=400, deadline=None)
@given(old=_template, new=_template)
def test_native_template_index_same_matches_the_guard(old, new):
    """`template_index_same` (the template store's index short-cut) equals comparing `_reference_guard`s."""
    from ncc.controller.controller import _reference_guard
    assert NATIVE.template_index_same(old, new) == (_reference_guard(old) == _reference_guard(new))
    assert NATIVE.template_index_same(old, old)
