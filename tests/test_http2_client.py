"""HTTP/2 in the Python clients (ncc/kube/h2client.py): the coordinator's connection to the controller cluster, and the
Python executor's to its shards, as client-go's transport speaks it (`/root/reference/main.go:52-68`).

* `RestClient(http2="on")` against the fake apiserver: CRUD, lists, error statuses, watches (lines, the line tap,
  a 410), all as streams of a few connections;
* negotiation: ALPN on TLS (`auto`, the default), and the fallbacks to HTTP/1.1 — a TLS server without h2 in its
  ALPN list, a cleartext server answering the preface in HTTP/1.1;
* the server's limits: MAX_CONCURRENT_STREAMS 4 (requests wait, or open a connection), a 64-byte stream window
  (request bodies wait for WINDOW_UPDATE), GOAWAY every 7 streams (the rest re-sent on a new connection), a header
  block larger than a frame (CONTINUATION), a request deadline (the stream reset, the connection kept);
* the native frame parser fed one byte at a time;
* the coordinator itself: an `App` over TLS reaches its controller apiserver over HTTP/2.
"""
import asyncio
import os

import pytest

from ncc import native
from ncc.fakeapi import native as fnative
from ncc.api import resources as R
from ncc.fakeapi.server import FakeApiServer
from ncc.kube import errors as E
from ncc.kube import h2client
from ncc.kube.kubeconfig import ClusterConfig, load_kubeconfig
from ncc.kube.rest import RestClient
from ncc.testing.env import FakeEnvironment
from ncc.testing.workload import make_configmap, make_secret, make_template

NS = "nexus"
_m = native.load(required=True)
_f = fnative.load(required=True)  # the fake apiserver's extension (server side)


class _Server:
    """A fake apiserver speaking HTTP/1.1 and HTTP/2 (prior knowledge) on cleartext."""

    async def __aenter__(self):
        self.srv = FakeApiServer(http2=True)
        return self.srv, await self.srv.start()

    async def __aexit__(self, *exc):
        await self.srv.stop()


async def test_rest_client_over_prior_knowledge_http2():
    async with _Server() as (srv, url):
        c = RestClient(ClusterConfig(server=url), http2="on")
        try:
            seen, tapped = [], []

            async def watch():
                async for lines in c.watch_raw_batches(R.SECRETS, NS, resource_version="0", on_lines=tapped.extend):
                    seen.extend(lines)
            w = asyncio.ensure_future(watch())
            await asyncio.gather(*[c.create(R.SECRETS, NS, make_secret(f"s{i}", NS)) for i in range(200)])
            assert c.protocol == "h2"
            got = await c.get(R.SECRETS, NS, "s7")
            got["data"] = {"k": "dmFsdWU="}
            assert (await c.update(R.SECRETS, NS, got))["data"] == {"k": "dmFsdWU="}
            assert len((await c.list(R.SECRETS, NS))["items"]) == 200
            with pytest.raises(E.NotFound):
                await c.get(R.SECRETS, NS, "missing")
            with pytest.raises(E.AlreadyExists):
                await c.create(R.SECRETS, NS, make_secret("s0", NS))
            # a 429 with Retry-After (the retry-after field of the response head): retried, then served
            srv.faults.update({"rules": [{"method": "PUT", "resource": "secrets", "code": 429, "count": 2,
                                          "retry_after": 0, "message": "slow down"}]})
            retries = c.stats["retries"]
            got = await c.get(R.SECRETS, NS, "s8")
            got["data"] = {"k": "dmFsdWU="}
            await c.update(R.SECRETS, NS, got)
            assert c.stats["retries"] == retries + 2
            await c.delete(R.SECRETS, NS, "s1")

            async def settled():
                return len(seen) >= 203
            for _ in range(200):
                if await settled():
                    break
                await asyncio.sleep(0.01)
            assert len(seen) == 203 and tapped == seen  # 200 ADDED, 2 MODIFIED, a DELETED; the tap saw each first
            w.cancel()
            st = srv._http.conn_stats()["h2"]
            # everything, the watch included, went over one connection (250 streams allowed on it)
            assert st["connections"] == 1 and st["streams"] >= 205, st
            assert c._pool.opened == 1
        finally:
            await c.close()


async def test_watch_errors_and_the_end_of_a_stream():
    async with _Server() as (srv, url):
        c = RestClient(ClusterConfig(server=url), http2="on")
        try:
            for i in range(3):
                await c.create(R.CONFIGMAPS, NS, make_configmap(f"c{i}", NS))
            lines = []
            async for batch in c.watch_raw_batches(R.CONFIGMAPS, NS, resource_version="0", timeout_seconds=1):
                lines.extend(batch)
            assert len(lines) == 3  # the server ended the stream after timeoutSeconds: the generator ends with it
            srv.state.compact()  # everything older is gone: a watch from resourceVersion 1 gets an ERROR event (410)
            got = []
            async for batch in c.watch_raw_batches(R.CONFIGMAPS, NS, resource_version="1"):
                got.extend(batch)
            assert len(got) == 1 and b'"ERROR"' in got[0] and b"410" in got[0], got
            with pytest.raises(E.NotFound):  # a watch answered with an error status
                async for _ in c.watch_raw_batches(R.ResourceType("nexus.example", "v1", "nothings", "Nothing"), NS):
                    pass
            assert c.protocol == "h2"
        finally:
            await c.close()


async def test_server_limits_windows_goaway_and_large_headers():
    async with _Server() as (srv, url):
        srv.faults.update({"h2_max_streams": 4, "h2_initial_window": 64})
        c = RestClient(ClusterConfig(server=url), http2="on", pool_size=2)
        try:
            await asyncio.gather(*[c.create(R.SECRETS, NS, make_secret(f"a{i}", NS)) for i in range(40)])
            st = srv._http.conn_stats()["h2"]
            # never more than 4 streams open on a connection (none refused), and at most the pool's 2 connections;
            # every 600-byte body went out in 64-byte pieces as the server's WINDOW_UPDATEs came
            assert st["max_open"] <= 4 and st["refused"] == 0 and 1 <= st["connections"] <= 2, st
        finally:
            await c.close()
        # a connection window of 64 KiB shared by 100 concurrent 600-byte bodies (credited as the server reads)
        srv.faults.update({"h2_max_streams": 0, "h2_initial_window": 0, "h2_small_conn_window": 1})
        c = RestClient(ClusterConfig(server=url), http2="on")
        try:
            big = [make_secret(f"w{i}", NS) for i in range(100)]
            for o in big:
                o["data"] = {"k": "A" * 4000}
            await asyncio.gather(*[c.create(R.SECRETS, NS, o) for o in big])
            assert srv.state.count(R.SECRETS, NS) == 140
        finally:
            await c.close()
        srv.faults.update({"h2_small_conn_window": 0, "h2_goaway_after": 7})
        c = RestClient(ClusterConfig(server=url, token="t" * 40000), http2="on")  # HEADERS + CONTINUATION
        try:
            await asyncio.gather(*[c.create(R.SECRETS, NS, make_secret(f"b{i}", NS)) for i in range(50)])
            assert srv.state.count(R.SECRETS, NS) == 190
            assert c._pool.stats["h2_goaways"] >= 5 and c._pool.opened >= 6, c._pool.stats
        finally:
            await c.close()


async def test_a_request_deadline_resets_the_stream_and_keeps_the_connection():
    async with _Server() as (srv, url):
        c = RestClient(ClusterConfig(server=url), http2="on", request_timeout=0.3, max_retries=0)
        try:
            await c.list(R.SECRETS, NS)
            srv.faults.update({"latency_ms": 2000})
            with pytest.raises(E.TransportError, match="timed out"):
                await c.list(R.SECRETS, NS)
            srv.faults.update({"latency_ms": 0})
            assert (await c.list(R.SECRETS, NS))["items"] == []
            assert c._pool.opened == 1  # the late stream was reset; its connection carried on
        finally:
            await c.close()


async def test_fallbacks_to_http11(tmp_path):
    async with _Server() as (srv, url):
        srv._http.http2 = False  # answers the prior-knowledge preface as HTTP/1.1 would
        c = RestClient(ClusterConfig(server=url), http2="on")
        try:
            await c.create(R.SECRETS, NS, make_secret("s0", NS))
            assert c.protocol == "http/1.1" and (await c.get(R.SECRETS, NS, "s0"))
            assert srv._http.conn_stats()["h2"]["connections"] == 0
        finally:
            await c.close()
        c = RestClient(ClusterConfig(server=url), http2="auto")  # cleartext + auto: HTTP/1.1 without trying
        try:
            await c.list(R.SECRETS, NS)
            assert c.protocol == "http/1.1"
        finally:
            await c.close()
        env = await FakeEnvironment(0, str(tmp_path), tls=True, http2=False).start()
        try:
            c = RestClient(load_kubeconfig(env.controller_kubeconfig))  # ALPN offers h2, the server picks http/1.1
            try:
                await c.list(R.SECRETS, NS)
                assert c.protocol == "http/1.1"
            finally:
                await c.close()
        finally:
            await env.stop()


async def test_coordinator_speaks_http2_to_a_tls_controller_apiserver(tmp_path):
    from ncc.app import App
    env = await FakeEnvironment(1, str(tmp_path), tls=True).start()
    cc = env.controller_client()
    stop, task = asyncio.Event(), None
    try:
        for i in range(5):
            await cc.create(R.SECRETS, NS, make_secret(f"s{i}", NS))
            await cc.create(R.CONFIGMAPS, NS, make_configmap(f"c{i}", NS))
            await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=[f"s{i}"], configmaps=[f"c{i}"]))
        app = App(env.app_config(mode="native", failure_rate_max_delay=0.2))
        await app.build()
        task = asyncio.ensure_future(app.run(stop))
        for _ in range(600):
            t = await cc.get(R.TEMPLATES, NS, "algo-00004")
            if ((t.get("status") or {}).get("conditions") or [{}])[0].get("status") == "True":
                break
            await asyncio.sleep(0.05)
        else:
            raise AssertionError("never Ready")
        client = app.client
        while not isinstance(client, type(cc)) and hasattr(client, "inner"):
            client = client.inner
        assert client.protocol == "h2"
        st = env.controller_server._http.conn_stats()["h2"]
        assert st["connections"] >= 1 and st["streams"] >= 10, st  # lists, watches, status writes, Events
    finally:
        stop.set()
        if task is not None:
            await task
        await cc.close()
        await env.stop()


def _frame(t, f, sid, p):
    return len(p).to_bytes(3, "big") + bytes([t, f]) + sid.to_bytes(4, "big") + p


def test_client_parser_from_any_framing():
    """Responses split over padded HEADERS, CONTINUATION and padded DATA, fed one byte at a time: one unary
    response, one watch's lines (a line across DATA frames; the trailing partial line at the end), control
    frames as events and the acks the connection owes written for it."""
    p = _m.H2ClientParser()
    p.watch(3)
    head = _m.hpack_encode([(":status", "200"), ("content-type", "application/json"), ("retry-after", "2")])
    frames = [_frame(4, 0, 0, (3).to_bytes(2, "big") + (100).to_bytes(4, "big")),
              _frame(1, 0x8, 1, bytes([2]) + head[:5] + b"\0\0"), _frame(9, 0x4, 1, head[5:]),
              _frame(0, 0x8, 1, bytes([1]) + b'{"a":' + b"\0"), _frame(0, 0x1, 1, b"1}"),
              _frame(1, 0x4, 3, _m.hpack_encode([(":status", "200")])),
              _frame(0, 0, 3, b'{"t":1}\n{"t"'), _frame(0, 0, 3, b':2}\n{"t":3'), _frame(0, 0x1, 3, b"}"),
              _frame(6, 0, 0, b"12345678"), _frame(8, 0, 0, (99).to_bytes(4, "big")),
              _frame(3, 0, 5, (7).to_bytes(4, "big")), _frame(7, 0, 0, (3).to_bytes(4, "big") + b"\0\0\0\0bye")]
    data = b"".join(frames)
    events, out = [], b""
    for i in range(len(data)):
        ev, o = p.feed(data[i:i + 1])
        events += ev
        out += o
    assert events[0] == ("settings", [(3, 100)])
    assert events[1] == ("resp", 1, 200, "2", b'{"a":1}')
    assert events[2] == ("head", 3, 200, None)
    lines = [ln for e in events if e[0] == "lines" for ln in e[2]]
    assert lines == [b'{"t":1}', b'{"t":2}', b'{"t":3}']
    assert [e for e in events if e[0] == "lines"][-1][4] is True
    assert events[-3:] == [("window", 0, 99), ("rst", 5, 7), ("goaway", 3, 0, b"bye")]
    assert out == _frame(4, 1, 0, b"") + _frame(6, 1, 0, b"12345678")  # SETTINGS ack, PING ack
    assert p.open_streams() == 0
    # a server that answers the preface in HTTP/1.1
    assert _m.H2ClientParser().feed(b"HTTP/1.1 400 Bad Request\r\n\r\n")[0] == [("noh2",)]
    # the request encoder: HEADERS split at the peer's frame size, DATA ending the stream
    fixed = _m.hpack_encode([(":scheme", "http"), (":authority", "a:1"), ("authorization", "x" * 100)])
    req = _m.h2_request(9, "PUT", "/api/v1/x", fixed, 5, b"hello", True, 64)
    d, off, kinds, block = _f.HpackDecoder(), 0, [], b""
    while off < len(req):
        n = int.from_bytes(req[off:off + 3], "big")
        kinds.append((req[off + 3], req[off + 4]))
        if req[off + 3] in (1, 9):
            block += req[off + 9:off + 9 + n]
        else:
            assert req[off + 9:off + 9 + n] == b"hello"
        off += 9 + n
    assert kinds[0] == (1, 0) and kinds[-2] == (9, 0x4) and kinds[-1] == (0, 0x1)
    assert d.decode(block) == [(":method", "PUT"), (":path", "/api/v1/x"), (":scheme", "http"),
                               (":authority", "a:1"), ("authorization", "x" * 100), ("content-length", "5")]
    assert h2client.AVAILABLE
    assert os.path.basename(h2client.__file__) == "h2client.py"


class Blackhole:
    """A TCP proxy whose connections can be frozen: from `freeze()` on, bytes already flowing through it are
    swallowed both ways while both sockets stay open — a path that died silently (a dropped NAT entry, a peer
    that lost power). Connections opened after the freeze pass normally."""

    def __init__(self, port: int):
        self.port, self.pairs, self.server = port, [], None

    async def start(self) -> str:
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        return f"http://127.0.0.1:{self.server.sockets[0].getsockname()[1]}"

    def freeze(self) -> None:
        for p in self.pairs:
            p["frozen"] = True

    async def _handle(self, r, w):
        ur, uw = await asyncio.open_connection("127.0.0.1", self.port)
        pair = {"frozen": False, "writers": (w, uw)}
        self.pairs.append(pair)

        async def pump(src, dst):
            try:
                while True:
                    data = await src.read(65536)
                    if not data:
                        break
                    if not pair["frozen"]:
                        dst.write(data)
            except (ConnectionError, asyncio.CancelledError):
                pass
            finally:
                if not pair["frozen"]:
                    dst.close()
        await asyncio.gather(pump(r, uw), pump(ur, w))

    async def stop(self) -> None:
        self.server.close()
        for p in self.pairs:
            for w in p["writers"]:
                w.close()


async def test_a_silent_connection_is_pinged_and_replaced(monkeypatch):
    """client-go's HTTP/2 health check: a connection that reads nothing for HTTP2_READ_IDLE_TIMEOUT_SECONDS while
    streams are open is PINGed, and dropped when HTTP2_PING_TIMEOUT_SECONDS pass without an answer. Its request
    fails at once rather than at its deadline, its watch ends (the informer re-watches), and the next request
    goes out on a new connection."""
    monkeypatch.setenv("HTTP2_READ_IDLE_TIMEOUT_SECONDS", "0.5")
    monkeypatch.setenv("HTTP2_PING_TIMEOUT_SECONDS", "0.5")
    async with _Server() as (srv, url):
        bh = Blackhole(int(url.rsplit(":", 1)[1]))
        purl = await bh.start()
        c = RestClient(ClusterConfig(server=purl), http2="on", request_timeout=20, max_retries=0)
        try:
            ended = asyncio.Event()

            async def watch():  # ends, or fails before its response head: either way the informer re-watches
                try:
                    async for _ in c.watch_raw_batches(R.CONFIGMAPS, NS, resource_version="0"):
                        pass
                except E.TransportError:
                    pass
                ended.set()
            w = asyncio.ensure_future(watch())
            assert (await c.list(R.SECRETS, NS))["items"] == []
            bh.freeze()
            loop = asyncio.get_running_loop()
            t0 = loop.time()
            with pytest.raises(E.TransportError, match="PING"):
                await c.list(R.SECRETS, NS)
            assert loop.time() - t0 < 5  # read-idle + PING timeout + sweep granularity, far below the 20 s deadline
            await asyncio.wait_for(ended.wait(), 5)
            await w
            assert (await c.list(R.SECRETS, NS))["items"] == []
            assert c._pool.stats["h2_dead"] == 1 and c._pool.opened == 2, c._pool.stats
        finally:
            await c.close()
            await bh.stop()


async def test_stream_resets_refusals_and_early_watch_exit():
    """A scripted HTTP/2 server (the native server parser and response encoder over a bare asyncio server):
    REFUSED_STREAM is retried (after a backoff) and then served; another reset code fails the request; a
    consumer that leaves a watch early resets its stream and the connection carries on; a malformed frame is a
    connection error (GOAWAY, the connection dropped) and the next request gets a new connection."""
    script = {"/refuse-once": ["refuse", "ok"], "/reset": ["reset"]}
    seen = []

    async def handle(reader, writer):
        parser = _f.H2ServerParser(False)
        writer.write(_frame(4, 0, 0, (3).to_bytes(2, "big") + (100).to_bytes(4, "big")) +
                     _frame(8, 0, 0, ((1 << 30) - 65535).to_bytes(4, "big")))
        while True:
            data = await reader.read(65536)
            if not data:
                break
            for ev in parser.feed(data):
                if ev[0] == "settings":
                    writer.write(_frame(4, 1, 0, b""))
                elif ev[0] == "req":
                    _, sid, method, path, headers, body = ev
                    seen.append((sid, path))
                    plan = script.get(path.split("?")[0])
                    step = plan.pop(0) if plan else "ok"
                    if step == "refuse":
                        writer.write(_frame(3, 0, sid, (7).to_bytes(4, "big")))
                    elif step == "reset":
                        writer.write(_frame(3, 0, sid, (2).to_bytes(4, "big")))
                    elif path == "/garbage":  # HEADERS on stream 0: a connection error
                        writer.write(_frame(1, 0x4, 0, b""))
                    elif "watch=1" in path:  # a watch: the head and two events, the stream left open
                        block = _m.hpack_encode([(":status", "200"), ("content-type", "application/json")])
                        writer.write(_frame(1, 0x4, sid, block) +
                                     _frame(0, 0, sid, b'{"type":"ADDED","object":{}}\n{"type":"ADDED","object":{}}\n'))
                    else:
                        writer.write(_f.h2_response(sid, 200, "application/json", b'{"kind":"SecretList","items":[]}',
                                                    [], 16384))
            await writer.drain()

    server = await asyncio.start_server(handle, "127.0.0.1", 0)
    url = f"http://127.0.0.1:{server.sockets[0].getsockname()[1]}"
    pool = h2client.H2Pool(url, prior_knowledge=True, connect_timeout=5)
    try:
        r = await pool.request("GET", "/refuse-once", {"Accept": "application/json"}, None, timeout=5)
        assert r.status == 200 and pool.stats["h2_refused"] == 1
        with pytest.raises(E.TransportError, match="reset by the server"):
            await pool.request("GET", "/reset", {"Accept": "application/json"}, None, timeout=5)
        got = []
        gen = pool.stream("/api/v1/namespaces/nexus/secrets?watch=1", {"Accept": "application/json"}, batch=True)
        async for resp, lines in gen:
            if resp is not None:
                assert resp.status == 200
                continue
            got.extend(lines)
            break  # leave early: the stream is reset, the connection stays
        await gen.aclose()
        assert len(got) == 2 and pool.conns and not pool.conns[0].streams
        assert (await pool.request("GET", "/after", {"Accept": "application/json"}, None, timeout=5)).status == 200
        assert pool.opened == 1
        with pytest.raises(E.TransportError, match="connection error"):
            await pool.request("GET", "/garbage", {"Accept": "application/json"}, None, timeout=5)
        assert (await pool.request("GET", "/after", {"Accept": "application/json"}, None, timeout=5)).status == 200
        assert pool.opened == 2  # the broken connection was closed (GOAWAY sent); a new one took over
    finally:
        pool.close()
        server.close()
        await server.wait_closed()


async def test_a_connection_whose_stream_ids_run_out_is_replaced():
    """Client stream ids are odd and below 2^31: a long-lived connection (≈ 7 h at 40 000 requests/s) runs out.
    The pool stops opening streams on it, moves to a new connection and closes the old one once drained."""
    async with _Server() as (srv, url):
        pool = h2client.H2Pool(url, prior_knowledge=True, connect_timeout=5)
        try:
            hdr = {"Accept": "application/json"}
            assert (await pool.request("GET", "/api/v1/namespaces/nexus/secrets", hdr, None)).status == 200
            first = pool.conns[0]
            first.next_sid = h2client.MAX_STREAM_ID - 2  # as after ~1e9 streams
            assert (await pool.request("GET", "/api/v1/namespaces/nexus/secrets", hdr, None)).status == 200
            assert first.draining and first.closed  # its last stream served, then closed
            assert (await pool.request("GET", "/api/v1/namespaces/nexus/configmaps", hdr, None)).status == 200
            assert pool.opened == 2 and pool.conns and pool.conns[0] is not first
        finally:
            pool.close()
