"""The lean HTTP/1.1 transport (`ncc.kube.transport`) and the REST client's credential/header fast paths,
against tiny raw asyncio servers (no fake apiserver), so framing, timeouts and slot accounting are
pinned independently of the control plane."""
import asyncio
import json
import time

import pytest

from ncc.kube import errors as E
from ncc.kube.kubeconfig import ClusterConfig, CredentialSource
from ncc.kube.rest import RestClient
from ncc.kube.transport import ConnectionPool


class _Server:
    """Minimal HTTP/1.1 server: answers each request with `handler(method, target, headers, body)`
    → (status, body bytes) or None (never answer)."""

    def __init__(self, handler):
        self.handler = handler
        self.requests = []
        self.server = None

    async def start(self) -> str:
        self.server = await asyncio.start_server(self._conn, "127.0.0.1", 0)
        return f"http://127.0.0.1:{self.server.sockets[0].getsockname()[1]}"

    async def _conn(self, reader, writer):
        try:
            while True:
                head = await reader.readuntil(b"\r\n\r\n")
                lines = head.decode("latin-1").split("\r\n")
                method, target, _ = lines[0].split(" ", 2)
                hdrs = {}
                for ln in lines[1:]:
                    if ln:
                        k, _, v = ln.partition(":")
                        hdrs[k.strip().lower()] = v.strip()
                body = await reader.readexactly(int(hdrs.get("content-length", "0")))
                self.requests.append((method, target, hdrs, body))
                res = await self.handler(method, target, hdrs, body)
                if res is None:
                    await asyncio.sleep(3600)
                status, out = res
                writer.write(b"HTTP/1.1 %d X\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
                             % (status, len(out), out))
                await writer.drain()
        except (asyncio.IncompleteReadError, ConnectionError, asyncio.CancelledError):
            pass
        finally:
            writer.close()

    async def stop(self):
        self.server.close()


async def test_pre_rendered_header_block_and_framing():
    async def ok(method, target, hdrs, body):
        return 200, json.dumps({"m": method, "t": target, "n": len(body)}).encode()
    srv = _Server(ok)
    url = await srv.start()
    pool = ConnectionPool(url, max_size=2)
    try:
        r = await pool.request("PUT", "/a?x=1", {"Accept": "application/json"}, b"{}",
                               block=b"Accept: application/json\r\nX-Pre: 1\r\n")
        assert r.status == 200 and json.loads(r.body) == {"m": "PUT", "t": "/a?x=1", "n": 2}
        _, _, hdrs, _ = srv.requests[-1]
        assert hdrs["x-pre"] == "1" and hdrs["content-length"] == "2" and hdrs["host"].startswith("127.0.0.1:")
        r = await pool.request("GET", "/b", {"Accept": "application/json"}, None)  # block rendered from the dict
        assert json.loads(r.body)["t"] == "/b" and "content-length" not in srv.requests[-1][2]
    finally:
        pool.close()
        await srv.stop()


async def test_request_timeout_is_swept_and_not_retried():
    calls = []

    async def hang(method, target, hdrs, body):
        calls.append(target)
        return None
    srv = _Server(hang)
    url = await srv.start()
    pool = ConnectionPool(url, max_size=2)
    pool.SWEEP_PERIOD = 0.05
    try:
        # warm the connection so the timed-out exchange runs on a reused one (the retry-once case)
        srv.handler = _ok_once(srv, hang)
        await pool.request("GET", "/warm", {}, None, timeout=5)
        loop = asyncio.get_running_loop()
        t0 = loop.time()
        with pytest.raises(E.TransportError, match="timed out"):
            await pool.request("POST", "/slow", {}, b"{}", timeout=0.2)
        assert 0.15 <= loop.time() - t0 < 2.0
        await asyncio.sleep(0.1)
        assert calls.count("/slow") == 1, "a timed-out request must not be re-sent"
        assert pool._inflight == 0
    finally:
        pool.close()
        await srv.stop()


def _ok_once(srv, then):
    state = {"n": 0}

    async def h(method, target, hdrs, body):
        state["n"] += 1
        if state["n"] == 1:
            return 200, b"{}"
        return await then(method, target, hdrs, body)
    return h


async def test_request_slots_bound_concurrency_and_survive_cancellation():
    live = {"now": 0, "max": 0}
    gate = asyncio.Event()

    async def slow(method, target, hdrs, body):
        live["now"] += 1
        live["max"] = max(live["max"], live["now"])
        await gate.wait()
        live["now"] -= 1
        return 200, b"{}"
    srv = _Server(slow)
    url = await srv.start()
    pool = ConnectionPool(url, max_size=2)
    try:
        tasks = [asyncio.ensure_future(pool.request("GET", f"/{i}", {}, None)) for i in range(8)]
        await asyncio.sleep(0.1)
        assert live["now"] == 2 and pool._inflight == 2 and len(pool._slot_waiters) == 6
        tasks[5].cancel()  # a waiter cancelled while queued gives nothing back and takes nothing
        await asyncio.sleep(0)
        gate.set()
        done = await asyncio.gather(*tasks, return_exceptions=True)
        assert isinstance(done[5], asyncio.CancelledError)
        assert all(getattr(r, "status", None) == 200 for i, r in enumerate(done) if i != 5)
        assert live["max"] == 2 and pool._inflight == 0 and not pool._slot_waiters
    finally:
        pool.close()
        await srv.stop()


async def test_file_token_is_cached_and_reread_after_period_or_401(tmp_path):
    tf = tmp_path / "token"
    tf.write_text("t1\n")
    cs = CredentialSource(ClusterConfig(server="http://x", token_file=str(tf)))
    assert cs.cached_token() == (False, None)  # never read yet
    assert await cs.token() == "t1"
    tf.write_text("t2\n")
    assert cs.cached_token() == (True, "t1") and await cs.token() == "t1"  # within the re-read period
    cs._file_read_at -= CredentialSource.FILE_TOKEN_PERIOD
    assert await cs.token() == "t2"

    seen = []

    async def auth(method, target, hdrs, body):
        seen.append(hdrs.get("authorization"))
        return (200, b"{}") if hdrs.get("authorization") == "Bearer t3" else (401, b'{"kind":"Status","code":401}')
    srv = _Server(auth)
    url = await srv.start()
    tf.write_text("t3\n")  # rotated: the cached t2 gets a 401, which forces one re-read
    c = RestClient(ClusterConfig(server=url, token_file=str(tf)))
    c.creds._file_token, c.creds._file_read_at = "t2", time.monotonic()
    try:
        assert await c.request("GET", "/api") == {}
        assert seen == ["Bearer t2", "Bearer t3"]
        await c.request("GET", "/api")
        assert seen[-1] == "Bearer t3" and len(c._hdr_cache) == 2  # (None, t2) and (None, t3)
    finally:
        await c.close()
        await srv.stop()


@pytest.mark.parametrize("head", [
    b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: 17",
    b"HTTP/1.1 201 Created\r\ncontent-length: 0\r\nConnection: close",
    b"HTTP/1.1 429 Too Many Requests\r\nRetry-After:  3 \r\nTransfer-Encoding: gzip, Chunked",
    b"HTTP/1.1 204 No Content",
    b"HTTP/1.0 503 Unavailable\r\nRetry-After: 1\r\nX-Other: a:b:c\r\nCONNECTION: Close",
])
def test_native_response_head_parser_matches_python(head):
    from ncc import native
    from ncc.kube.transport import _parse_head_py
    m = native.load(required=True)
    status, clen, chunked, close, retry = m.parse_response_head(head)
    ps, pc, pch, pcl, ph = _parse_head_py(head)
    assert (status, clen, chunked, close, retry) == (ps, pc, pch, pcl, ph.get("retry-after"))


@pytest.mark.parametrize("head", [b"garbage", b"HTTP/1.1 2x0 OK", b"HTTP/1.1 200 OK\r\nContent-Length: -5"])
def test_native_response_head_parser_rejects_malformed(head):
    from ncc import native
    with pytest.raises(ValueError):
        native.load(required=True).parse_response_head(head)


def test_native_request_head_parser_matches_python():
    from ncc.fakeapi import native as fnative
    from ncc.fakeapi.httpserver import _parse_head_py
    m = fnative.load(required=True)
    for head in (b"PUT /api/v1/namespaces/n/secrets/a?fieldManager=x HTTP/1.1\r\nHost: h:1\r\nContent-Length: 12",
                 b"GET /apis/x/y?watch=1 HTTP/1.1\r\nAuthorization:  Bearer t \r\nX-Odd: a: b\r\nNoColonLine",
                 b"DELETE /a HTTP/1.1"):
        assert m.parse_request_head(head) == _parse_head_py(head)
    for bad in (b"GARBAGE", b"GET /only-two", b" / HTTP/1.1"):
        with pytest.raises(ValueError):
            m.parse_request_head(bad)


async def test_pipelined_responses_in_one_read_and_split_reads():
    """Several responses in one TCP read (pipelining) and a response split over reads both frame right."""
    from ncc.kube.transport import _Conn

    class _Pool:
        pipeline_depth = 4

        def _release(self, c):
            pass

        def _discard(self, c):
            pass

    loop = asyncio.get_running_loop()
    c = _Conn(_Pool())
    futs = [loop.create_future() for _ in range(3)]
    c.pending.extend(futs)
    r = lambda b: b"HTTP/1.1 200 OK\r\nContent-Length: %d\r\n\r\n%s" % (len(b), b)  # noqa: E731
    c.data_received(r(b'{"a":1}') + r(b"") + r(b'{"c":3}')[:20])
    assert futs[0].result().body == b'{"a":1}' and futs[1].result().body == b"" and not futs[2].done()
    c.data_received(r(b'{"c":3}')[20:])
    assert futs[2].result().body == b'{"c":3}'


async def test_watch_batches_drain_lines_that_arrive_during_processing():
    """Lines that arrive while the consumer is busy with a batch are delivered before the stream ends."""
    async def handler(reader, writer):
        await reader.readuntil(b"\r\n\r\n")
        writer.write(b"HTTP/1.1 200 OK\r\nTransfer-Encoding: chunked\r\n\r\n")
        for i in range(5):
            line = b'{"n":%d}\n' % i
            writer.write(b"%x\r\n%s\r\n" % (len(line), line))
            await writer.drain()
            await asyncio.sleep(0.01)
        writer.write(b"0\r\n\r\n")
        await writer.drain()
        writer.close()
    srv = await asyncio.start_server(handler, "127.0.0.1", 0)
    url = f"http://127.0.0.1:{srv.sockets[0].getsockname()[1]}"
    pool = ConnectionPool(url)
    got = []
    try:
        async for resp, lines in pool.stream("/w?watch=1", {}, batch=True):
            if resp is not None:
                continue
            got.extend(lines)
            await asyncio.sleep(0.05)  # slow consumer: later lines and the end of the stream arrive meanwhile
        assert got == [b'{"n":%d}' % i for i in range(5)]
    finally:
        pool.close()
        srv.close()


def test_native_parsers_survive_arbitrary_bytes():
    """Random and truncated inputs: the C++ parsers return or raise ValueError, never crash."""
    from hypothesis import given, settings, strategies as st
    from ncc import native
    from ncc.fakeapi import native as fnative
    m = native.load(required=True)
    f = fnative.load(required=True)  # the fake apiserver's request-head parser
    good_resp = b"HTTP/1.1 200 OK\r\nContent-Length: 5\r\nRetry-After: 1"
    good_req = b"PUT /api/v1/namespaces/n/secrets/a HTTP/1.1\r\nContent-Length: 3"
    good_line = (b'{"type":"MODIFIED","object":{"metadata":{"name":"s","namespace":"n","resourceVersion":"7",'
                 b'"ownerReferences":[{"name":"t","uid":"u"}]}}}')

    flt, idx = m.OwnerFilter(), m.RelayIndex()  # their memos persist across the examples

    @settings(max_examples=300, deadline=None)
    @given(st.binary(max_size=200), st.integers(0, 200))
    def check(blob, cut):
        for fn in (m.parse_response_head, f.parse_request_head):
            for data in (blob, good_resp[:cut] + blob, good_req[:cut] + blob):
                try:
                    fn(data)
                except ValueError:
                    pass
        for data in (blob, good_line[:cut], good_line[:cut] + blob):
            r = m.scan_event_part(data, 3, "n")
            assert r is None or len(r) == 8
            m.scan_event_owners(data)
            m.scan_object(data)
            kept, dropped, _ = m.owner_filter([data], {("n", "s"): {"metadata": {"ownerReferences": []}}}, {}, "n")
            assert len(kept) + dropped == 1
            assert m.relay_index([data], {}, "n") in ([], [data])
            kept, dropped, _ = flt([data], {("n", "s"): {"metadata": {"ownerReferences": []}}}, {}, "n")
            assert len(kept) + dropped == 1
            assert idx([data], {}, "n") in ([], [data])
            try:  # undecodable text (not UTF-8) raises ValueError, as json.loads does
                m.template_event_slim(data, {("n", "s"): {"status": {}, "__ncc_sfp__": 1}}, "n")
            except ValueError:
                pass
            try:
                m.chunk_lines(bytearray(data), -1, bytearray())
            except ValueError:
                pass
    check()


async def test_write_meta_fast_path_errors_and_retries():
    """write_meta's direct-to-pool path: a 2xx is scanned natively; a 409 raises Conflict; a 429 with
    Retry-After is retried through the general exchange loop."""
    from ncc.api import resources as R
    seq = []

    async def handler(method, target, hdrs, body):
        seq.append((method, target))
        n = len(seq)
        if n == 1:
            return 200, b'{"metadata":{"namespace":"n","name":"a","resourceVersion":"7","uid":"u1"}}'
        if n == 2:
            return 409, b'{"kind":"Status","code":409,"reason":"Conflict","message":"modified"}'
        if n == 3:
            return 429, b'{"kind":"Status","code":429}'
        return 201, b'{"metadata":{"namespace":"n","name":"b","resourceVersion":"9","uid":"u2"}}'

    class RetrySrv(_Server):
        async def _conn(self, reader, writer):
            try:
                while True:
                    head = await reader.readuntil(b"\r\n\r\n")
                    lines = head.decode("latin-1").split("\r\n")
                    method, target, _ = lines[0].split(" ", 2)
                    hdrs = {ln.partition(":")[0].strip().lower(): ln.partition(":")[2].strip() for ln in lines[1:] if ln}
                    body = await reader.readexactly(int(hdrs.get("content-length", "0")))
                    status, out = await self.handler(method, target, hdrs, body)
                    extra = b"Retry-After: 0\r\n" if status == 429 else b""
                    writer.write(b"HTTP/1.1 %d X\r\n%sContent-Length: %d\r\n\r\n%s" % (status, extra, len(out), out))
                    await writer.drain()
            except (asyncio.IncompleteReadError, ConnectionError):
                pass
            finally:
                writer.close()

    srv = RetrySrv(handler)
    url = await srv.start()
    c = RestClient(ClusterConfig(server=url))
    try:
        await c._get_pool()
        assert await c.write_meta("update", R.SECRETS, "n", {"metadata": {"name": "a"}}, name="a") == \
            ("n", "a", "7", "u1")
        with pytest.raises(E.Conflict):
            await c.write_meta("update", R.SECRETS, "n", {"metadata": {"name": "a"}}, name="a")
        assert await c.write_meta("create", R.SECRETS, "n", {"metadata": {"name": "b"}}) == ("n", "b", "9", "u2")
        assert [m for m, _ in seq] == ["PUT", "PUT", "POST", "POST"] and c.stats["retries"] == 1
    finally:
        await c.close()
        await srv.stop()


def _python_stream_lines(body: bytes, cuts: list[int]) -> tuple[list, bool]:
    """The Python chunked-stream path (`_parse_chunks` + `_feed_stream`) fed `body` in the given pieces."""
    from ncc.kube import transport as T
    saved, T._chunk_lines = T._chunk_lines, None
    try:
        return _stream_lines(body, cuts)
    finally:
        T._chunk_lines = saved


def _stream_lines(body: bytes, cuts: list[int]) -> tuple[list, bool]:
    from collections import deque
    from ncc.kube.transport import _Conn

    class _Pool:
        pipeline_depth = 1

    c = _Conn(_Pool())
    c.stream, c.stream_event, c.head_done, c.chunked = deque(), asyncio.Event(), True, True
    done = False
    prev = 0
    for cut in sorted(set(cuts)) + [len(body)]:
        c.buf += body[prev:cut]
        prev = cut
        done = c._parse_chunks() or done
        if done:
            break
    return list(c.stream), done


def test_native_chunk_lines_match_the_python_path():
    """The native splitter yields the same lines, in any split of the bytes, as the Python path, and the
    same end-of-body verdict; malformed chunk framing raises ValueError."""
    from hypothesis import given, settings, strategies as st
    from ncc import native
    from ncc.kube import transport as T
    native.load(required=True)
    assert T._chunk_lines is not None

    @settings(max_examples=300, deadline=None)
    @given(st.lists(st.binary(min_size=1, max_size=40), max_size=8), st.lists(st.integers(0, 400), max_size=6),
           st.booleans())
    def check(pieces, cuts, ext):
        body = b"".join(b"%x%s\r\n%s\r\n" % (len(p), b";x=1" if ext else b"", p) for p in pieces) + b"0\r\nT: v\r\n\r\n"
        cuts = [c for c in cuts if c < len(body)]
        assert _stream_lines(body, cuts) == _python_stream_lines(body, cuts)
    check()
    lines, done = _stream_lines(b"5\r\n{\"a\":\r\n4\r\n1}\n\n\r\n0\r\n\r\n", [3, 9])
    assert lines == [b'{"a":1}'] and done
    m = native.load(required=True)
    for bad in (b"zz\r\n", b"3\r\nabcXY"):
        with pytest.raises(ValueError):
            m.chunk_lines(bytearray(bad), -1, bytearray())


def test_native_relay_index_matches_relay_scan():
    """relay_index (the one-partition relay loop) stores, deletes and forwards exactly what a relay_scan loop
    does."""
    from ncc import native
    m = native.load(required=True)

    def ev(t, name, ns="n"):
        return json.dumps({"type": t, "object": {"metadata": {"name": name, "namespace": ns,
                                                              "resourceVersion": "1"}}}).encode()
    lines = [ev("ADDED", "a"), ev("MODIFIED", "b", ""), ev("BOOKMARK", "c"), b"garbage", ev("DELETED", "a"),
             ev("DELETED", "zz"), ev("ADDED", "d"), ev("ERROR", "e")]
    raw_py, keep_py = {("n", "old"): b"x"}, []
    for line in lines:
        sc = m.relay_scan(line, 1, "dflt")
        if sc is None or sc[0] == 3:
            continue
        if sc[0] == 2:
            raw_py.pop((sc[1], sc[2]), None)
        else:
            raw_py[(sc[1], sc[2])] = line
        keep_py.append(line)
    raw = {("n", "old"): b"x"}
    assert m.relay_index(lines, raw, "dflt") == keep_py
    assert raw == raw_py and ("dflt", "b") in raw


def test_native_owner_filter_matches_the_python_filter():
    """owner_filter drops exactly the MODIFIED lines of cached, non-overlaid objects whose owner names and uids
    equal the cached ones (the metadata-only informer's Python filter), and reports the last dropped RV."""
    from ncc import native
    m = native.load(required=True)

    def line(t, name, owners, ns="n", rv="5"):
        md = {"name": name, "namespace": ns, "resourceVersion": rv}
        if owners is not None:
            md["ownerReferences"] = [{"apiVersion": "v1", "kind": "T", "name": o, "uid": u} for o, u in owners]
        return json.dumps({"type": t, "object": {"metadata": md, "data": {"k": "v"}}}, ensure_ascii=False).encode()

    def cached(owners):
        md = {"name": "x"}
        if owners is not None:
            md["ownerReferences"] = [{"name": o, "uid": u} for o, u in owners]
        return {"metadata": md}
    items = {("n", "a"): cached([("t1", "u1")]), ("n", "b"): cached(None), ("n", "c"): cached([("t1", "u1")]),
             ("n", "d"): cached([("t1", "u1"), ("t2", "u2")]), ("n", "e"): cached([]), ("n", "é"): cached([("t", "ü")])}
    assumed = {("n", "c"): None}
    lines = [line("MODIFIED", "a", [("t1", "u1")], rv="10"),       # same owners: dropped
             line("MODIFIED", "a", [("t1", "u9")], rv="11"),       # uid changed: kept
             line("MODIFIED", "b", None, rv="12"),                 # no owners either side: dropped
             line("MODIFIED", "c", [("t1", "u1")], rv="13"),       # overlaid: kept
             line("MODIFIED", "d", [("t2", "u2"), ("t1", "u1")]),  # order differs: kept
             line("ADDED", "a", [("t1", "u1")]),                   # not MODIFIED: kept
             line("MODIFIED", "zz", None),                         # not cached: kept
             b"garbage",
             line("MODIFIED", "e", None, rv="14"),                 # [] vs none: dropped
             line("MODIFIED", "é", [("t", "ü")], rv="15")]         # UTF-8 names: dropped
    kept, dropped, last = m.owner_filter(lines, items, assumed, "n")
    assert dropped == 4 and last == "15"
    assert kept == [lines[i] for i in (1, 3, 4, 5, 6, 7)]
    kept, dropped, last = m.owner_filter(lines[:2], items, assumed, "n")
    assert dropped == 1 and last is None and kept == [lines[1]]


def test_memoising_owner_filter_matches_owner_filter():
    """OwnerFilter (the informer's per-store memo) gives owner_filter's result batch after batch while the store's
    objects are replaced, overlaid and deleted under it; a replaced object is compared by its new owners."""
    import random
    from ncc import native
    m = native.load(required=True)
    rnd = random.Random(7)

    def line(t, name, owners, rv):
        md = {"name": name, "namespace": "n", "resourceVersion": str(rv)}
        if owners is not None:
            md["ownerReferences"] = [{"apiVersion": "v1", "kind": "T", "name": o, "uid": u} for o, u in owners]
        return json.dumps({"type": t, "object": {"metadata": md, "data": {"k": "v"}}}).encode()

    owner_sets = [None, [], [("t1", "u1")], [("t1", "u2")], [("t1", "u1"), ("t2", "u2")]]
    names = [f"o{i}" for i in range(12)]
    items: dict = {}
    assumed: dict = {}
    flt = m.OwnerFilter()
    rv = 0
    for _ in range(300):
        for _ in range(rnd.randint(0, 4)):  # the store changes between batches
            name = rnd.choice(names)
            op = rnd.random()
            if op < 0.5:
                o = owner_sets[rnd.randrange(len(owner_sets))]
                md = {"name": name} if o is None else {"name": name, "ownerReferences": [{"name": a, "uid": b}
                                                                                         for a, b in o]}
                items[("n", name)] = {"metadata": md}
            elif op < 0.7:
                items.pop(("n", name), None)
            elif op < 0.85:
                assumed[("n", name)] = None
            else:
                assumed.pop(("n", name), None)
        batch = []
        for _ in range(rnd.randint(1, 6)):
            rv += 1
            batch.append(line(rnd.choice(["MODIFIED", "MODIFIED", "ADDED"]), rnd.choice(names),
                              owner_sets[rnd.randrange(len(owner_sets))], rv))
        assert flt(list(batch), items, assumed, "n") == m.owner_filter(list(batch), items, assumed, "n")
    assert 0 < len(flt) <= len(names)
    flt.clear()
    assert len(flt) == 0


def test_memoising_owner_filter_keeps_a_bounded_memo():
    """Deleted keys do not accumulate: the memo is dropped whole once it outgrows the store by 4096 keys."""
    from ncc import native
    m = native.load(required=True)
    flt = m.OwnerFilter()
    for i in range(5000):
        key = ("n", f"x{i}")
        items = {key: {"metadata": {"name": key[1]}}}
        line = json.dumps({"type": "MODIFIED", "object": {"metadata": {"name": key[1], "resourceVersion": str(i)}}})
        kept, dropped, last = flt([line.encode()], items, {}, "n")
        assert dropped == 1 and last == str(i) and kept == []
    assert len(flt) <= 4098


def test_memoising_relay_index_matches_relay_index():
    """RelayIndex (the relay's per-kind memo of key tuples) indexes and forwards exactly as relay_index, batch
    after batch, through deletes, re-creates and a `raw` dict swapped for a relist."""
    import random
    from ncc import native
    m = native.load(required=True)
    rnd = random.Random(11)
    names = [f"o{i}" for i in range(10)] + ["é"]
    idx = m.RelayIndex()
    raw_a: dict = {}
    raw_b: dict = {}
    for step in range(400):
        batch = []
        for _ in range(rnd.randint(1, 6)):
            t = rnd.choice(["ADDED", "MODIFIED", "MODIFIED", "DELETED", "BOOKMARK"])
            ns = rnd.choice(["", "n"])
            batch.append(json.dumps({"type": t, "object": {"metadata": {"name": rnd.choice(names), "namespace": ns,
                                                                        "resourceVersion": str(step)}}}).encode())
        if rnd.random() < 0.05:
            batch.append(b"not json")
        assert idx(list(batch), raw_a, "dflt") == m.relay_index(list(batch), raw_b, "dflt")
        assert raw_a == raw_b
        if step == 200:  # a relist swaps the dict
            raw_a, raw_b = dict(raw_a), dict(raw_b)
    assert len(idx) <= len(names) * 2


def test_native_sampler_records_and_hands_the_signal_on(tmp_path):
    """NCC_NATIVE_SAMPLE's sampler (native/ext/sampler.hpp): installed in front of a Python SIGPROF handler, it
    records the interrupted instruction and still lets the Python handler run; the dump holds the executable
    mappings and one "pc tos" line per sample."""
    import signal
    from ncc import native
    m = native.load(required=True)
    hits = [0]
    old = signal.signal(signal.SIGPROF, lambda *_: hits.__setitem__(0, hits[0] + 1))
    signal.setitimer(signal.ITIMER_PROF, 0.0005, 0.0005)
    try:
        assert m.native_sample_start(500)
        objs = [{"k": list(range(200)), "s": "x" * 500}] * 200
        deadline = time.process_time() + 1.0
        while time.process_time() < deadline and hits[0] < 20:
            m.fingerprint_many(objs)
        path = tmp_path / "native.samples"
        n = m.native_sample_dump(str(path))
    finally:
        signal.setitimer(signal.ITIMER_PROF, 0, 0)
        signal.signal(signal.SIGPROF, old)
    assert hits[0] > 0  # the Python handler still ran
    text = path.read_text()
    assert "# map " in text
    rows = [ln for ln in text.splitlines() if ln and not ln.startswith("#")]
    assert len(rows) == n and n > 0 and all(len(r.split()) == 2 for r in rows)
