"""HTTP/2 between the C++ shard executor (native/executor/h2.hpp) and the fake apiserver (ncc/fakeapi/h2.py).

client-go speaks HTTP/2 to kube-apiservers — negotiated by ALPN on TLS — and multiplexes a clientset's requests
on one connection (`/root/reference/main.go:52-68`).  `client-http2` gives the C++ executor the same: `auto`
(the default) where TLS negotiates it, `on` also with prior knowledge on cleartext.

* HPACK (native/common/hpack.hpp) against RFC 7541 Appendix C — the request examples without and with Huffman
  coding (C.3, C.4) and the response examples with eviction from a 256-byte table (C.5) — and round trips.
* The executor over HTTP/2 against the same scenarios as HTTP/1.1: cold sync, updates, few connections carrying
  many streams; TLS with ALPN; GOAWAY mid-run (streams past the last one re-sent on a new connection); a
  MAX_CONCURRENT_STREAMS of 4 (more connections, never more streams than allowed); a 64-byte stream window
  (request bodies wait for WINDOW_UPDATE); a header block larger than a frame (CONTINUATION).
"""
import asyncio
import os
import random

import pytest

from ncc import native
from ncc.fakeapi import native as fnative
from ncc.api import resources as R
from ncc.testing.workload import make_configmap, make_secret, make_template

from test_conformance import NS, Cluster, mutate, wait_for

_m = native.load(required=True)
_f = fnative.load(required=True)  # the fake apiserver's extension (server side)


# ---------------------------------------------------------------------------------------------- HPACK
C3 = ["828684410f7777772e6578616d706c652e636f6d",
      "828684be58086e6f2d6361636865",
      "828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565"]
C4 = ["828684418cf1e3c2e5f23a6ba0ab90f4ff",
      "828684be5886a8eb10649cbf",
      "828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf"]
C3_FIELDS = [
    [(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com")],
    [(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com"),
     ("cache-control", "no-cache")],
    [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"), (":authority", "www.example.com"),
     ("custom-key", "custom-value")]]
C5 = ["4803333032580770726976617465611d4d6f6e2c203231204f637420323031332032303a31333a323120474d546e1768747470733a2f2f"
      "7777772e6578616d706c652e636f6d",
      "4803333037c1c0bf",
      "88c1611d4d6f6e2c203231204f637420323031332032303a31333a323220474d54c05a04677a69707738666f6f3d4153444a4b48514b"
      "425a584f5157454f50495541585157454f49553b206d61782d6167653d333630303b2076657273696f6e3d31"]


@pytest.mark.parametrize("blocks", [C3, C4], ids=["C.3-plain", "C.4-huffman"])
def test_hpack_rfc7541_request_examples(blocks):
    d = _f.HpackDecoder(4096)
    sizes = []
    for blk, want in zip(blocks, C3_FIELDS):
        assert d.decode(bytes.fromhex(blk)) == want
        sizes.append(d.table_size())
    assert sizes == [57, 110, 164]  # the dynamic table sizes the RFC lists after each request


def test_hpack_rfc7541_response_examples_with_eviction():
    d = _f.HpackDecoder(256)
    got = [d.decode(bytes.fromhex(b)) for b in C5[:1]]
    assert got[0] == [(":status", "302"), ("cache-control", "private"), ("date", "Mon, 21 Oct 2013 20:13:21 GMT"),
                      ("location", "https://www.example.com")]
    assert d.table_size() == 222
    assert d.decode(bytes.fromhex(C5[1]))[0] == (":status", "307")
    assert d.table_size() == 222 and d.table_entries() == 4  # ":status: 302" evicted for ":status: 307"
    third = d.decode(bytes.fromhex(C5[2]))
    assert third[-1] == ("set-cookie", "foo=ASDJKHQKBZXOQWEOPIUAXQWEOIU; max-age=3600; version=1")
    assert d.table_size() == 215 and d.table_entries() == 3


def test_hpack_huffman_rfc_strings_and_round_trip():
    for s, h in ((b"www.example.com", "f1e3c2e5f23a6ba0ab90f4ff"), (b"no-cache", "a8eb10649cbf"),
                 (b"custom-key", "25a849e95ba97d7f"), (b"custom-value", "25a849e95bb8e8b4bf")):
        assert _m.hpack_huffman_encode(s).hex() == h
        assert _m.hpack_huffman_decode(bytes.fromhex(h)) == s
    rnd = random.Random(7)
    for _ in range(300):
        s = bytes(rnd.randrange(256) for _ in range(rnd.randrange(0, 64)))
        assert _m.hpack_huffman_decode(_m.hpack_huffman_encode(s)) == s
    with pytest.raises(ValueError):
        _m.hpack_huffman_decode(b"\xff\xff\xff\xff")  # EOS inside a string


def test_hpack_encoder_round_trip_and_malformed_blocks():
    rnd = random.Random(3)
    d = _f.HpackDecoder()
    for _ in range(100):
        fields = [(":status", str(rnd.choice([200, 201, 404, 409, 429, 503]))), ("content-type", "application/json")]
        fields += [(f"x-{rnd.randrange(1000)}", "v" * rnd.randrange(0, 300)) for _ in range(rnd.randrange(4))]
        for huff in (False, True):
            assert d.decode(_m.hpack_encode(fields, huff)) == fields
    assert d.table_size() == 0  # literals without indexing never touch the table
    for bad in (b"\x80", b"\xff\xff\xff\xff\xff\xff\xff\xff\xff\xff\x7f", b"\x40\x05ab", b"\xbe"):
        with pytest.raises(ValueError):
            d.decode(bad)
    fresh = _f.HpackDecoder()
    with pytest.raises(ValueError):  # a table size update after a field
        fresh.decode(bytes.fromhex("82") + b"\x20")
    with pytest.raises(ValueError):  # above the limit we advertised
        fresh.decode(b"\x3f\xe2\x1f")  # 4097


# ---------------------------------------------------------------------------------------------- the executor
@pytest.fixture
def native_only():
    from ncc.controller.native_executor import binary_path
    if binary_path() is None:
        pytest.skip("ncc/bin/ncc-executor is not built")


def _flow(cl) -> dict:
    ex = cl.app.debug_state().get("executors") or {}
    out = {}
    for h in ex.values():
        out.update((h.get("status") or {}).get("flow") or {})
    return out


async def _converge(cl, n: int, tag: str = ""):
    async def ok():
        for s in cl.sstates:
            for i in range(n):
                t = s.try_get(R.TEMPLATES, NS, f"algo-{i:05d}")
                if t is None or (tag and t["spec"]["container"]["versionTag"] != tag):
                    return False
                if s.try_get(R.CONFIGMAPS, NS, f"c{i}") is None or s.try_get(R.SECRETS, NS, f"s{i}") is None:
                    return False
        return True
    await wait_for(ok, timeout=30, interval=0.05)
    for i in range(n):
        await cl.ready(f"algo-{i:05d}")


async def _h2_status(cl):
    async def ok():
        fl = _flow(cl)
        return bool(fl) and all(f.get("http2") == 1 and f.get("h2_streams", 0) > 0 for f in fl.values()) and fl
    return await wait_for(ok, timeout=10, interval=0.1)


async def test_executor_syncs_over_http2_prior_knowledge(tmp_path, native_only, monkeypatch):
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    async with Cluster(tmp_path, "native", n_shards=2, client_http2="on", executors_per_shard=1) as cl:
        n = 30
        for i in range(n):
            cl.seed(i, secrets=(f"s{i}",), configmaps=(f"c{i}",))
        await cl.start()
        await _converge(cl, n)
        for i in range(n):
            await mutate(cl.cc, R.TEMPLATES, f"algo-{i:05d}",
                         lambda o: o["spec"]["container"].__setitem__("versionTag", "h2v"))
        await _converge(cl, n, "h2v")
        fl = await _h2_status(cl)
        for i, srv in enumerate(cl.env.shard_servers):
            st = srv._http.conn_stats()
            # every write and list of the executor went over a few HTTP/2 connections
            assert st["h2"]["connections"] >= 1 and st["h2"]["streams"] >= 2 * n, st
            assert st["h2"]["connections"] <= 2, st
            assert fl[f"shard-{i}"]["connections"] <= 2, fl
            # the executor's four watches are streams on the same connection: nothing else is open to the shard
            assert st["open"] <= 2, st
            assert srv.requests["watch_streams"] >= 4
            assert st["h2"]["malformed"] == 0, st  # every header block well-formed (pseudo-headers first)
        assert all(f["rejected_429"] == 0 for f in fl.values())
        # client-pool-size auto: an HTTP/2 shard may have 1024 requests in flight (streams, not connections)
        from ncc.controller.native_executor import DEFAULT_H2_INFLIGHT
        assert all(f["cap"] == DEFAULT_H2_INFLIGHT for f in fl.values()), fl
        # the same flow status as per-shard gauges (statsd / Prometheus)
        from ncc.api import constants as C
        from ncc.telemetry.statsd import MemoryMetrics
        cl.app.metrics = MemoryMetrics()
        cl.app._gauges()
        v = cl.app.metrics.values
        assert v[C.SHARD_CLIENT_METRICS["http2"]] == [1.0, 1.0], v
        assert all(x >= 1 for x in v[C.SHARD_CLIENT_METRICS["limit"]]) and len(v[C.SHARD_CLIENT_METRICS["limit"]]) == 2
        assert v[C.SHARD_CLIENT_METRICS["rejected_429"]] == [0.0, 0.0]
        assert v[C.SHARD_CLIENT_METRICS["cap"]] == [float(DEFAULT_H2_INFLIGHT)] * 2, v


async def test_explicit_pool_size_caps_http2_too(tmp_path, native_only, monkeypatch):
    """An explicit client-pool-size is the in-flight cap over HTTP/2 as over HTTP/1.1 (no 1024-stream default)."""
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    async with Cluster(tmp_path, "native", n_shards=1, client_http2="on", client_pool_size=8,
                       executors_per_shard=1) as cl:
        for i in range(10):
            cl.seed(i, secrets=(f"s{i}",), configmaps=(f"c{i}",))
        await cl.start()
        await _converge(cl, 10)
        fl = await _h2_status(cl)
        assert fl["shard-0"]["cap"] == 8 and fl["shard-0"]["max_inflight"] <= 8, fl


async def test_executor_negotiates_http2_by_alpn_on_tls(tmp_path, native_only, monkeypatch):
    """`client-http2: auto` (the default): on TLS the executor offers "h2" and the server selects it."""
    from ncc.app import App
    from ncc.testing.env import FakeEnvironment
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    env = await FakeEnvironment(1, str(tmp_path), tls=True).start()
    cc, sc = env.controller_client(), env.shard_client(0)
    app, stop, task = None, asyncio.Event(), None
    try:
        for i in range(5):
            await cc.create(R.SECRETS, NS, make_secret(f"s{i}", NS))
            await cc.create(R.CONFIGMAPS, NS, make_configmap(f"c{i}", NS))
            await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=[f"s{i}"], configmaps=[f"c{i}"]))
        app = App(env.app_config(mode="native", executor_impl="native", failure_rate_max_delay=0.2))
        await app.build()
        task = asyncio.ensure_future(app.run(stop))

        async def ready():
            for i in range(5):
                t = await cc.get(R.TEMPLATES, NS, f"algo-{i:05d}")
                c = (t.get("status") or {}).get("conditions") or [{}]
                if c[0].get("status") != "True":
                    return False
            return True
        await wait_for(ready, timeout=30, interval=0.05)
        st = env.shard_servers[0]._http.conn_stats()
        assert st["h2"]["connections"] >= 1 and st["h2"]["streams"] >= 15, st
        assert (await sc.get(R.SECRETS, NS, "s4"))["metadata"]["ownerReferences"]
    finally:
        stop.set()
        if task is not None:
            await task
        await cc.close()
        await sc.close()
        await env.stop()


async def test_goaway_mid_run_moves_streams_to_a_new_connection(tmp_path, native_only, monkeypatch):
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    async with Cluster(tmp_path, "native", n_shards=1, client_http2="on", executors_per_shard=1) as cl:
        cl.env.shard_servers[0].faults.update({"h2_goaway_after": 7})
        n = 20
        for i in range(n):
            cl.seed(i, secrets=(f"s{i}",), configmaps=(f"c{i}",))
        await cl.start()
        await _converge(cl, n)
        st = cl.env.shard_servers[0]._http.conn_stats()["h2"]
        assert st["goaways"] >= 3 and st["connections"] >= 4, st  # ≥ 3·n writes, 7 streams per connection
        await _h2_status(cl)

        async def saw_goaway():  # (the status messages come every 0.2 s)
            fl = _flow(cl)
            return fl.get("shard-0", {}).get("h2_goaways", 0) >= 1
        await wait_for(saw_goaway, timeout=5, interval=0.1)


async def test_stream_limit_is_obeyed_and_small_windows_hold_bodies(tmp_path, native_only, monkeypatch):
    """MAX_CONCURRENT_STREAMS 4: the executor never has more streams open on a connection (the server refuses
    any extra with REFUSED_STREAM — none come) and opens more connections; a 64-byte stream window and a
    connection window left at 65 535 make every request body wait for the server's WINDOW_UPDATEs."""
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    async with Cluster(tmp_path, "native", n_shards=1, client_http2="on", executors_per_shard=1,
                       client_pool_size=8) as cl:
        cl.env.shard_servers[0].faults.update({"h2_max_streams": 4, "h2_initial_window": 64,
                                               "h2_small_conn_window": 1})
        n = 25
        for i in range(n):
            cl.seed(i, secrets=(f"s{i}",), configmaps=(f"c{i}",))
        await cl.start()
        await _converge(cl, n)
        st = cl.env.shard_servers[0]._http.conn_stats()["h2"]
        assert st["max_open"] <= 4 and st["refused"] == 0, st
        assert 1 <= st["connections"] <= 8, st
        fl = await _h2_status(cl)
        assert fl["shard-0"]["h2_refused"] == 0, fl


async def test_large_header_block_goes_out_in_continuation_frames(tmp_path, native_only, monkeypatch):
    """A 40 kB bearer token (an OIDC token with many groups can be that large) makes the header block longer
    than a 16 kB frame: HEADERS + CONTINUATION."""
    from ncc.app import App
    from ncc.testing.env import FakeEnvironment
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    token = "t" * 40000
    env = await FakeEnvironment(1, str(tmp_path), token=token).start()
    cc = env.controller_client()
    stop, task = asyncio.Event(), None
    try:
        await cc.create(R.SECRETS, NS, make_secret("s0", NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap("c0", NS))
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=["s0"], configmaps=["c0"]))
        app = App(env.app_config(mode="native", executor_impl="native", client_http2="on",
                                 failure_rate_max_delay=0.2))
        await app.build()
        task = asyncio.ensure_future(app.run(stop))

        async def synced():
            return env.shard_servers[0].state.try_get(R.CONFIGMAPS, NS, "c0") is not None
        await wait_for(synced, timeout=30, interval=0.05)
        st = env.shard_servers[0]._http.conn_stats()["h2"]
        assert st["streams"] >= 3, st
    finally:
        stop.set()
        if task is not None:
            await task
        await cc.close()
        await env.stop()


async def test_http2_off_and_a_server_without_h2_fall_back_to_http11(tmp_path, native_only, monkeypatch):
    """`client-http2: off` never speaks it; `auto` on TLS against a server that does not offer h2 in ALPN
    carries on over HTTP/1.1."""
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    async with Cluster(tmp_path, "native", n_shards=1, client_http2="off", executors_per_shard=1) as cl:
        cl.seed(0)
        await cl.start()
        await cl.ready()
        assert cl.env.shard_servers[0]._http.conn_stats()["h2"]["connections"] == 0
    # `on` against a cleartext server that answers the preface in HTTP/1.1: the executor falls back
    async with Cluster(tmp_path / "h1only", "native", n_shards=1, client_http2="on", executors_per_shard=1) as cl:
        cl.env.shard_servers[0]._http.http2 = False
        cl.seed(0)
        await cl.start()
        await cl.ready()
        assert cl.env.shard_servers[0]._http.conn_stats()["h2"]["connections"] == 0

        async def h1_flow():  # back to HTTP/1.1: the in-flight cap is the pool again, not the HTTP/2 cap
            fl = _flow(cl).get("shard-0") or {}
            return fl.get("http2") == 0 and fl.get("requests", 0) > 0 and fl
        from ncc.controller.native_executor import DEFAULT_POOL_SIZE
        fl = await wait_for(h1_flow, timeout=5, interval=0.1)
        assert fl["cap"] == DEFAULT_POOL_SIZE and fl["limit"] <= DEFAULT_POOL_SIZE, fl
    from ncc.app import App
    from ncc.testing.env import FakeEnvironment
    os.makedirs(tmp_path / "tls", exist_ok=True)
    env = await FakeEnvironment(1, str(tmp_path / "tls"), tls=True, http2=False).start()
    cc = env.controller_client()
    stop, task = asyncio.Event(), None
    try:
        await cc.create(R.SECRETS, NS, make_secret("s0", NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap("c0", NS))
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=["s0"], configmaps=["c0"]))
        app = App(env.app_config(mode="native", executor_impl="native", failure_rate_max_delay=0.2))
        await app.build()
        task = asyncio.ensure_future(app.run(stop))

        async def synced():
            return env.shard_servers[0].state.try_get(R.CONFIGMAPS, NS, "c0") is not None
        await wait_for(synced, timeout=30, interval=0.05)
        assert env.shard_servers[0]._http.conn_stats()["h2"]["connections"] == 0

        async def h1_cap():  # ALPN chose http/1.1: the cap is the pool (256), not the HTTP/2 cap
            ex = app.debug_state().get("executors") or {}
            fl = [(h.get("status") or {}).get("flow", {}).get("shard-0") for h in ex.values()]
            fl = [f for f in fl if f and f.get("http2") == 0 and f.get("requests", 0) > 0]
            return fl and fl[0]
        from ncc.controller.native_executor import DEFAULT_POOL_SIZE
        fl = await wait_for(h1_cap, timeout=5, interval=0.1)
        assert fl["cap"] == DEFAULT_POOL_SIZE, fl
    finally:
        stop.set()
        if task is not None:
            await task
        await cc.close()
        await env.stop()


def test_server_parser_assembles_streams_from_any_framing():
    """The fake apiserver's native frame parser (ncc/fakeapi/h2.py): a request split over HEADERS with padding
    and priority, CONTINUATION and padded DATA frames, fed one byte at a time, comes out as one request;
    control frames come out as events; a broken preface is a connection error."""
    from ncc.fakeapi import h2
    block = _m.hpack_encode([(":method", "PUT"), (":scheme", "http"), (":authority", "a:1"),
                             (":path", "/api/v1/namespaces/n/configmaps/c"), ("content-type", "application/json")])
    first, rest = block[:10], block[10:]
    pad = 3
    frames = [h2.PREFACE, h2.frame(h2.SETTINGS, 0, 0, bytes.fromhex("000400010000")),
              h2.frame(h2.HEADERS, h2.PADDED | h2.PRIORITY_FLAG, 1, bytes([pad]) + b"\0\0\0\0\x10" + first + b"\0" * pad),
              h2.frame(h2.CONTINUATION, h2.END_HEADERS, 1, rest),
              h2.frame(h2.DATA, h2.PADDED, 1, bytes([2]) + b'{"a":' + b"\0\0"),
              h2.frame(h2.DATA, h2.END_STREAM, 1, b"1}"),
              h2.frame(h2.WINDOW_UPDATE, 0, 0, (1000).to_bytes(4, "big")),
              h2.frame(h2.PING, 0, 0, b"12345678"), h2.frame(h2.RST_STREAM, 0, 3, (8).to_bytes(4, "big"))]
    data = b"".join(frames)
    p = _f.H2ServerParser(False)
    events = []
    for i in range(len(data)):
        events += p.feed(data[i:i + 1])
    assert events[0] == ("settings", [(4, 65536)])
    kind, sid, method, path, headers, body = events[1]
    assert (kind, sid, method, path, body) == ("req", 1, "PUT", "/api/v1/namespaces/n/configmaps/c", b'{"a":1}')
    assert headers == {"content-type": "application/json", "host": "a:1"}
    assert events[2:] == [("window", 0, 1000), ("ping", b"12345678"), ("rst", 3, 8)]
    assert p.open_streams() == 0
    bad = _f.H2ServerParser(False)
    assert bad.feed(b"GET / HTTP/1.1\r\nHost: x\r\n\r\n")[0][0] == "error"
    # the connection window is given back as request bodies use it (a soak once stalled after 1 GiB of them)
    cp = _f.H2ServerParser(False, 1000)
    hdr = h2.frame(h2.HEADERS, h2.END_HEADERS, 1, block)
    ev = cp.feed(h2.PREFACE + hdr + b"".join(h2.frame(h2.DATA, 0, 1, b"x" * 600) for _ in range(3)))
    assert ("credit", 0, 1200) in ev and [e for e in ev if e[0] == "credit"] == [("credit", 0, 1200)]
    resp = _f.h2_response(5, 200, "application/json", b"x" * 40000, [("retry-after", "1")], 16384)
    d = _f.HpackDecoder()
    n = int.from_bytes(resp[:3], "big")
    assert resp[3] == h2.HEADERS and resp[4] == h2.END_HEADERS
    assert d.decode(resp[9:9 + n]) == [(":status", "200"), ("content-type", "application/json"),
                                       ("content-length", "40000"), ("retry-after", "1")]
    off, got, flags = 9 + n, b"", []
    while off < len(resp):
        n = int.from_bytes(resp[off:off + 3], "big")
        flags.append(resp[off + 4])
        got += resp[off + 9:off + 9 + n]
        off += 9 + n
    assert got == b"x" * 40000 and flags == [0, 0, h2.END_STREAM]
    # a pseudo-header after a regular field is a malformed request (RFC 9113 §8.3): Go's server, and this one,
    # reset that stream and keep the connection
    late = _m.hpack_encode([(":method", "GET"), (":scheme", "http"), ("user-agent", "x"), (":path", "/api")])
    mp = _f.H2ServerParser(False)
    ev = mp.feed(h2.PREFACE + h2.frame(h2.HEADERS, h2.END_HEADERS | h2.END_STREAM, 1, late)
                 + h2.frame(h2.HEADERS, h2.END_HEADERS | h2.END_STREAM, 3, block))
    assert ev[0] == ("malformed", 1) and ev[1][:2] == ("req", 3) and mp.open_streams() == 0
    no_path = _m.hpack_encode([(":method", "GET"), (":scheme", "http"), (":authority", "a:1")])
    assert mp.feed(h2.frame(h2.HEADERS, h2.END_HEADERS | h2.END_STREAM, 5, no_path)) == [("malformed", 5)]
    upper = _m.hpack_encode([(":method", "GET"), (":scheme", "http"), (":path", "/"), ("User-Agent", "x")])
    assert mp.feed(h2.frame(h2.HEADERS, h2.END_HEADERS | h2.END_STREAM, 7, upper)) == [("malformed", 7)]


async def test_a_silent_shard_connection_is_pinged_and_replaced(tmp_path, native_only, monkeypatch):
    """The C++ executor's HTTP/2 health check (client-go's HTTP2_READ_IDLE_TIMEOUT_SECONDS and
    HTTP2_PING_TIMEOUT_SECONDS): the path to shard-0 goes silent mid-run — bytes swallowed both ways, sockets
    open. Without the check the next writes would wait out their 30 s deadline and be re-sent on the same dead
    connection; with it the connection is PINGed, dropped, and the writes and watches move to a new one."""
    from test_http2_client import Blackhole
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    monkeypatch.setenv("HTTP2_READ_IDLE_TIMEOUT_SECONDS", "1")
    monkeypatch.setenv("HTTP2_PING_TIMEOUT_SECONDS", "1")
    async with Cluster(tmp_path, "native", n_shards=1, client_http2="on", executors_per_shard=1) as cl:
        bh = Blackhole(int(cl.env.shard_servers[0].url.rsplit(":", 1)[1]))
        purl = await bh.start()
        with open(os.path.join(cl.env.shard_dir, "shard-0.kubeconfig"), "w") as f:
            f.write(cl.env.kubeconfig(purl, "shard-0"))
        try:
            n = 5
            for i in range(n):
                cl.seed(i, secrets=(f"s{i}",), configmaps=(f"c{i}",))
            await cl.start()
            await _converge(cl, n)
            bh.freeze()
            t0 = asyncio.get_running_loop().time()
            for i in range(n):
                await mutate(cl.cc, R.TEMPLATES, f"algo-{i:05d}",
                             lambda o: o["spec"]["container"].__setitem__("versionTag", "after"))
            await _converge(cl, n, "after")
            assert asyncio.get_running_loop().time() - t0 < 15

            async def dropped():
                return _flow(cl).get("shard-0", {}).get("h2_dead", 0) >= 1
            await wait_for(dropped, timeout=5, interval=0.1)
        finally:
            await bh.stop()
