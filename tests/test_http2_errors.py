"""HTTP/2 error codes in both shard/controller clients ("next 3"), against a scripted server.

Each behaviour runs for the Python pool (`ncc/kube/h2client.py` `H2Pool`, the coordinator's transport) and for the
C++ executor's client (`native/executor/http.hpp`, driven by the test tool `build/tools/ncc-h2probe`, which compiles
the same header):

* a GOAWAY with an error code (ENHANCE_YOUR_CALM) backs the re-send of the streams it refused off (≥ 50 ms), and
  counts; one with NO_ERROR does not count as an error;
* HTTP_1_1_REQUIRED in RST_STREAM or in GOAWAY moves the client to HTTP/1.1: the refused request is served over
  HTTP/1.1 and so is every later one, with a warning;
* WINDOW_UPDATE of 0, and one pushing a window past 2^31-1: a stream error (RST_STREAM PROTOCOL_ERROR /
  FLOW_CONTROL_ERROR) on a stream, a connection error (GOAWAY with that code, then close) on the connection;
* a server whose SETTINGS_HEADER_TABLE_SIZE is 0 (it limits *our* encoder) and which indexes its response fields
  in its own 4096-byte table: both decoders keep that table;
* the in-flight cap: over HTTP/2 the C++ client keeps up to `h2_cap` requests in flight on `pool` connections, and
  falls back to pool × depth when the shard moves to HTTP/1.1;
* framing: padded HEADERS/DATA and PRIORITY fields, a header block split over CONTINUATION frames are read; a pad
  length past its frame, a header block interrupted by another frame, and a CONTINUATION without HEADERS are
  connection errors (GOAWAY PROTOCOL_ERROR, then a new connection).

Reference behaviour being matched: client-go's HTTP/2 transport (Go's x/net/http2), /root/reference/main.go:52-68.
"""
import asyncio
import json
import os
import sys
import time

import pytest

from ncc import native
from ncc.fakeapi import native as fnative
from ncc.kube import errors as E
from ncc.kube import h2client

_m = native.load(required=True)
_f = fnative.load(required=True)  # the fake apiserver's extension: the scripted server's framing
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"
HDR = {"Accept": "application/json"}
OK_BODY = b'{"kind":"Status","status":"Success"}'


def _frame(t, f, sid, p=b""):
    return len(p).to_bytes(3, "big") + bytes([t, f]) + (sid & 0x7FFFFFFF).to_bytes(4, "big") + p


def _goaway(last, code, debug=b""):
    return _frame(7, 0, 0, last.to_bytes(4, "big") + code.to_bytes(4, "big") + debug)


def _server_parser():
    return _f.H2ServerParser(False)


def probe_path():
    sys.path.insert(0, os.path.join(ROOT, "native"))
    import build
    try:
        return build.build_tools()
    except Exception as e:  # noqa: BLE001 — no compiler / libssl: the C++ cases skip
        pytest.skip(f"ncc-h2probe not buildable here: {e}")


class Scripted:
    """An HTTP/2 (prior knowledge) and HTTP/1.1 server.  `script[path]` is a list of actions, one per request to
    that path (then "ok"); every frame the clients send that matters here is recorded in `seen`."""

    def __init__(self, script: dict, settings: list | None = None):
        self.script = {k: list(v) for k, v in script.items()}
        self.settings = settings or [(3, 100)]
        self.seen = []  # (time, kind, ...) — "req" (proto, path, sid), "rst" (sid, code), "goaway" (last, code)
        self.server = None
        self.h2 = True  # False: answer the HTTP/2 preface as an HTTP/1.1-only server does

    def log(self, *ev):
        self.seen.append((time.monotonic(), *ev))

    def of(self, kind):
        return [e[1:] for e in self.seen if e[1] == kind]

    async def start(self) -> str:
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        return f"http://127.0.0.1:{self.server.sockets[0].getsockname()[1]}"

    async def stop(self):
        self.server.close()
        await self.server.wait_closed()

    async def _handle(self, reader, writer):
        try:
            head = await reader.readexactly(24)
        except asyncio.IncompleteReadError:
            writer.close()
            return
        try:
            if head == PREFACE and self.h2:
                await self._h2(reader, writer)
            else:
                await self._h1(head, reader, writer)
        except (ConnectionError, asyncio.IncompleteReadError):
            pass
        finally:
            writer.close()

    async def _h1(self, head, reader, writer):
        buf = head
        while True:
            while b"\r\n\r\n" not in buf:
                chunk = await reader.read(65536)
                if not chunk:
                    return
                buf += chunk
            hdr, _, buf = buf.partition(b"\r\n\r\n")
            lines = hdr.decode().split("\r\n")
            method, path, _ = lines[0].split(" ", 2)
            clen = 0
            for ln in lines[1:]:
                k, _, v = ln.partition(":")
                if k.strip().lower() == "content-length":
                    clen = int(v.strip())
            while len(buf) < clen:
                buf += await reader.read(65536)
            buf = buf[clen:]
            self.log("req", "http/1.1", path, 0)
            if path == "/slow":
                await asyncio.sleep(0.05)
            writer.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\n\r\n%s"
                         % (len(OK_BODY), OK_BODY))
            await writer.drain()

    async def _h2(self, reader, writer):
        parser = _server_parser()
        st = b"".join(k.to_bytes(2, "big") + v.to_bytes(4, "big") for k, v in self.settings)
        writer.write(_frame(4, 0, 0, st))
        parser.feed(PREFACE)
        while True:
            data = await reader.read(65536)
            if not data:
                return
            for ev in parser.feed(data):
                kind = ev[0]
                if kind == "settings":
                    writer.write(_frame(4, 1, 0))
                elif kind == "rst":
                    self.log("rst", ev[1], ev[2])
                elif kind == "goaway":
                    self.log("goaway", ev[1], ev[2])
                elif kind == "req":
                    _, sid, method, path, headers, body = ev
                    path = path.split("?")[0]
                    self.log("req", "h2", path, sid)
                    plan = self.script.get(path)
                    action = plan.pop(0) if plan else "ok"
                    last = sid - 2 if sid > 1 else 0
                    if action == "ok" and path == "/slow":  # answered 200 ms later, the connection serving others
                        asyncio.get_running_loop().call_later(
                            0.2, writer.write, _f.h2_response(sid, 200, "application/json", OK_BODY, [], 16384))
                    elif action == "ok":
                        writer.write(_f.h2_response(sid, 200, "application/json", OK_BODY, [], 16384))
                    elif action == "goaway_calm":  # ENHANCE_YOUR_CALM: this stream refused
                        writer.write(_goaway(last, 0xB, b"too many requests"))
                        await writer.drain()
                        self.log("sent_goaway", 0xB)
                        return
                    elif action == "goaway_ok":
                        writer.write(_goaway(last, 0))
                        await writer.drain()
                        return
                    elif action == "goaway_h11":
                        writer.write(_goaway(last, 0xD))
                        await writer.drain()
                        return
                    elif action == "rst_h11":
                        writer.write(_frame(3, 0, sid, (0xD).to_bytes(4, "big")))
                    elif action == "win0_stream":
                        writer.write(_frame(8, 0, sid, (0).to_bytes(4, "big")))
                    elif action == "win0_conn":
                        writer.write(_frame(8, 0, 0, (0).to_bytes(4, "big")))
                    elif action == "winmax_stream":
                        writer.write(_frame(8, 0, sid, (0x7FFFFFFF).to_bytes(4, "big")))
                    elif action == "winmax_conn":
                        writer.write(_frame(8, 0, 0, (0x7FFFFFFF).to_bytes(4, "big")))
                    elif action == "padded":  # HEADERS with PADDED + PRIORITY, DATA with PADDED: legal framing
                        hdr = b"\x03" + b"\x00\x00\x00\x00\x10" + b"\x88" + b"\x00" * 3
                        data = b"\x05" + OK_BODY + b"\x00" * 5
                        writer.write(_frame(1, 0x4 | 0x8 | 0x20, sid, hdr) + _frame(0, 0x1 | 0x8, sid, data))
                    elif action == "continuation":  # a header block split over HEADERS + CONTINUATION
                        block = b"\x88" + b"\x40\x06x-test\x03abc"
                        writer.write(_frame(1, 0, sid, block[:4]) + _frame(9, 0, sid, block[4:9]) +
                                     _frame(9, 0x4, sid, block[9:]) + _frame(0, 0x1, sid, OK_BODY))
                    elif action == "bad_padding":  # a pad length past the frame: PROTOCOL_ERROR (RFC 9113 6.1)
                        writer.write(_frame(1, 0x4, sid, b"\x88") + _frame(0, 0x1 | 0x8, sid, b"\x40" + OK_BODY))
                    elif action == "interrupted":  # a header block interrupted by another frame (RFC 9113 6.10)
                        writer.write(_frame(1, 0, sid, b"\x88") + _frame(0, 0x1, sid, OK_BODY))
                    elif action == "lone_continuation":  # CONTINUATION without HEADERS
                        writer.write(_frame(9, 0x4, sid, b"\x88"))
                    elif action == "indexed":
                        # our fields indexed in the server's own (4096-byte) dynamic table, whatever
                        # SETTINGS_HEADER_TABLE_SIZE the client sent or we sent
                        block = b"\x88" + b"\x40\x06x-test\x03abc" if not getattr(self, "_indexed", False) \
                            else b"\x88\xbe"
                        self._indexed = True
                        writer.write(_frame(1, 0x4, sid, block) + _frame(0, 0x1, sid, OK_BODY))
            await writer.drain()


async def py_requests(url, paths, **kw):
    pool = h2client.H2Pool(url, prior_knowledge=True, connect_timeout=5, **kw)
    out = []
    try:
        for p in paths:
            try:
                r = await pool.request("GET", p, HDR, None, timeout=5)
                out.append({"status": r.status, "t": time.monotonic()})
            except E.TransportError as e:
                out.append({"error": str(e), "t": time.monotonic()})
        return out, dict(pool.stats, protocol=pool.protocol)
    finally:
        pool.close()


async def cpp_requests(url, paths, steps=None, args=()):
    probe = probe_path()
    steps = steps if steps is not None else "".join(f"GET {p}\nWAIT\n" for p in paths)
    proc = await asyncio.create_subprocess_exec(probe, url, "2", "--timeout", "5", *args, stdin=asyncio.subprocess.PIPE,
                                                stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE)
    t0 = time.monotonic()
    out, err = await asyncio.wait_for(proc.communicate(steps.encode()), 60)
    lines = [json.loads(x) for x in out.decode().splitlines() if x.strip()]
    assert lines and "stats" in lines[-1], (out, err)
    res = sorted(lines[:-1], key=lambda r: r["i"])
    for r in res:
        r["t"] = t0 + r["ms"] / 1000.0
    stats = dict(lines[-1]["stats"], notices=lines[-1]["notices"])
    stats["protocol"] = "h2" if stats["http2"] else "http/1.1"
    return res, stats


CLIENTS = {"python": py_requests, "cpp": cpp_requests}


@pytest.mark.parametrize("client", sorted(CLIENTS))
async def test_goaway_error_code_backs_off_the_resend(client):
    srv = Scripted({"/calm": ["goaway_calm"], "/bye": ["goaway_ok"]})
    url = await srv.start()
    try:
        res, stats = await CLIENTS[client](url, ["/calm", "/bye", "/after"])
        assert [r.get("status") for r in res] == [200, 200, 200], res
        reqs = srv.of("req")
        calm = [e for e in srv.seen if e[1] in ("sent_goaway", "req") and (e[1] == "sent_goaway" or e[3] == "/calm")]
        t_goaway = next(e[0] for e in calm if e[1] == "sent_goaway")
        t_retry = [e[0] for e in calm if e[1] == "req"][1]
        assert t_retry - t_goaway >= 0.045, "the refused stream was re-sent without backing off"
        assert [r[2] for r in reqs].count("/calm") == 2 and [r[2] for r in reqs].count("/bye") == 2
        assert stats["h2_goaway_errors"] == 1 and stats["h2_goaways"] == 2 and stats["protocol"] == "h2"
        if client == "cpp":
            assert any("GOAWAY with HTTP/2 error 11" in n for n in stats["notices"])
    finally:
        await srv.stop()


@pytest.mark.parametrize("how", ["rst_h11", "goaway_h11"])
@pytest.mark.parametrize("client", sorted(CLIENTS))
async def test_http_1_1_required_downgrades(client, how):
    srv = Scripted({"/x": [how]})
    url = await srv.start()
    try:
        res, stats = await CLIENTS[client](url, ["/x", "/y"])
        assert [r.get("status") for r in res] == [200, 200], res
        reqs = srv.of("req")
        assert [(r[1], r[2]) for r in reqs] == [("h2", "/x"), ("http/1.1", "/x"), ("http/1.1", "/y")], reqs
        assert stats["h2_downgraded"] == 1 and stats["protocol"] == "http/1.1"
        if client == "cpp":
            assert any("requires HTTP/1.1" in n for n in stats["notices"])
    finally:
        await srv.stop()


@pytest.mark.parametrize("client", sorted(CLIENTS))
@pytest.mark.parametrize("action,code", [("win0_stream", 1), ("winmax_stream", 3)])
async def test_bad_stream_window_update_is_a_stream_error(client, action, code):
    srv = Scripted({"/w": [action]})
    url = await srv.start()
    try:
        res, stats = await CLIENTS[client](url, ["/w", "/after"])
        assert srv.of("rst") and srv.of("rst")[0][2] == code, srv.seen  # RST_STREAM with the right code
        assert not srv.of("goaway")  # the connection carries on
        assert res[-1].get("status") == 200
        if client == "python":
            assert "stream error" in res[0]["error"]
        else:  # the C++ client re-sends a failed exchange once; the script serves the second
            assert res[0].get("status") == 200
        assert len({r[3] for r in srv.of("req")}) == len(srv.of("req"))  # distinct streams, one connection
    finally:
        await srv.stop()


@pytest.mark.parametrize("client", sorted(CLIENTS))
@pytest.mark.parametrize("action,code", [("win0_conn", 1), ("winmax_conn", 3)])
async def test_bad_connection_window_update_is_a_connection_error(client, action, code):
    srv = Scripted({"/w": [action]})
    url = await srv.start()
    try:
        res, stats = await CLIENTS[client](url, ["/w", "/after"])
        goaways = srv.of("goaway")
        assert goaways and goaways[0][2] == code, srv.seen  # GOAWAY sent before the close, with the error code
        assert res[-1].get("status") == 200  # a new connection serves what follows
        if client == "python":
            assert "connection error" in res[0]["error"]
    finally:
        await srv.stop()


@pytest.mark.parametrize("client", sorted(CLIENTS))
async def test_server_header_table_size_zero_keeps_our_decoder_table(client):
    srv = Scripted({"/i": ["indexed", "indexed"]}, settings=[(1, 0), (3, 100)])
    url = await srv.start()
    try:
        res, stats = await CLIENTS[client](url, ["/i", "/i"])
        assert [r.get("status") for r in res] == [200, 200], res
        assert not srv.of("goaway"), srv.seen  # no COMPRESSION_ERROR
    finally:
        await srv.stop()


async def test_pool_falls_back_per_connection_after_speaking_http2():
    """a connection that no longer negotiates HTTP/2 after earlier ones did (a load balancer with mixed
    backends, a server downgraded) moves the pool to HTTP/1.1 instead of failing for good, as Go's transport
    decides per connection."""
    srv = Scripted({})
    url = await srv.start()
    pool = h2client.H2Pool(url, prior_knowledge=True, connect_timeout=5)
    try:
        assert (await pool.request("GET", "/a", HDR, None, timeout=5)).status == 200 and pool.protocol == "h2"
        srv.h2 = False
        for c in list(pool.conns):
            c.abort("test: the backend changed")
        await asyncio.sleep(0.05)
        assert (await pool.request("GET", "/b", HDR, None, timeout=5)).status == 200
        assert pool.protocol == "http/1.1" and pool.opened == 1
        assert [(r[1], r[2]) for r in srv.of("req")][-1] == ("http/1.1", "/b")
    finally:
        pool.close()
        await srv.stop()


@pytest.mark.parametrize("client", sorted(CLIENTS))
@pytest.mark.parametrize("action", ["padded", "continuation"])
async def test_legal_framing_variants_are_read(client, action):
    srv = Scripted({"/f": [action]})
    url = await srv.start()
    try:
        res, stats = await CLIENTS[client](url, ["/f", "/after"])
        assert [r.get("status") for r in res] == [200, 200], res
        assert not srv.of("goaway") and not srv.of("rst"), srv.seen
        assert len(srv.of("req")) == 2  # nothing re-sent
    finally:
        await srv.stop()


@pytest.mark.parametrize("client", sorted(CLIENTS))
@pytest.mark.parametrize("action", ["bad_padding", "interrupted", "lone_continuation"])
async def test_framing_violations_are_connection_errors(client, action):
    srv = Scripted({"/f": [action]})
    url = await srv.start()
    try:
        res, stats = await CLIENTS[client](url, ["/f", "/after"])
        goaways = srv.of("goaway")
        assert goaways and goaways[0][2] == 1, srv.seen  # GOAWAY(PROTOCOL_ERROR) before the close
        assert res[-1].get("status") == 200  # a new connection serves what follows
    finally:
        await srv.stop()


async def test_cpp_http2_inflight_cap_and_its_fallback():
    """`h2_cap` (coordinator `DEFAULT_H2_INFLIGHT` when client-pool-size is auto): over HTTP/2, 12 slow requests
    run 8 at a time on a pool of 2 connections; once the shard requires HTTP/1.1, the cap is pool × depth (2) again."""
    srv = Scripted({})
    url = await srv.start()
    try:
        steps = "GET /slow\n" * 12 + "WAIT\n"
        res, stats = await cpp_requests(url, None, steps, ("--pool", "2", "--h2-cap", "8"))
        assert [r.get("status") for r in res] == [200] * 12, res
        assert stats["protocol"] == "h2" and stats["cap"] == 8 and stats["max_inflight"] == 8, stats
        assert stats["connections"] <= 2
        assert 0.35 <= max(r["ms"] for r in res) / 1000.0 < 1.5  # two rounds of 200 ms, not six
        # control: no h2 cap -> pool x depth over HTTP/2 too
        res, stats = await cpp_requests(url, None, steps, ("--pool", "2"))
        assert stats["cap"] == 2 and stats["max_inflight"] == 2, stats
    finally:
        await srv.stop()
    srv = Scripted({"/x": ["rst_h11"]})
    url = await srv.start()
    try:
        steps = "GET /x\nWAIT\n" + "GET /slow\n" * 12 + "WAIT\n"
        res, stats = await cpp_requests(url, None, steps, ("--pool", "2", "--h2-cap", "8"))
        assert [r.get("status") for r in res] == [200] * 13, res
        assert stats["protocol"] == "http/1.1" and stats["h2_downgraded"] == 1
        assert stats["cap"] == 2 and stats["max_inflight"] <= 2, stats
        assert {r[1] for r in srv.of("req") if r[2] == "/slow"} == {"http/1.1"}
    finally:
        await srv.stop()
