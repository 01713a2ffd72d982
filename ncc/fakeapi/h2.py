"""HTTP/2 (RFC 9113) for the fake kube-apiserver: the server side of the shard executor's HTTP/2 client.

client-go talks to kube-apiservers over HTTP/2 — ALPN "h2" on TLS — multiplexing every request of a clientset
on one connection (`/root/reference/main.go:52-68` builds the clients; Go's transport negotiates h2).  The
C++ shard executor does the same with `client-http2` (native/executor/h2.hpp); this module lets the fake
apiserver answer it, so the HTTP/2 path runs against the same substrate as everything else:

* negotiation: ALPN "h2" on a TLS connection (`--http2` puts it in the server's ALPN list), or the client
  connection preface on a cleartext one ("prior knowledge", how the benches and tests run it unencrypted);
* one `H2Connection` per connection on top of `httpserver._ServerConn`: frames parsed, streams assembled and
  HPACK decoded as they arrive by the extension's `H2ServerParser` (native/common/hpack.hpp, one dynamic table
  per connection), each complete stream handed to the same handlers as an HTTP/1.1 request — concurrently,
  as streams are; a response that fits the windows is framed natively in one call (`h2_response`);
* responses as HEADERS + DATA within the client's flow-control windows (connection and stream), queued
  until a WINDOW_UPDATE when they do not fit; watch streams as DATA frames without END_STREAM;
* SETTINGS (MAX_CONCURRENT_STREAMS enforced with REFUSED_STREAM), PING, RST_STREAM, WINDOW_UPDATE, GOAWAY.

Fault knobs (`POST /_fake/faults`), for connections opened afterwards: `h2_goaway_after` — after that many
streams a connection sends GOAWAY naming the last stream it will serve, and refuses later ones (a
kube-apiserver does this on shutdown and, with `--goaway-chance`, to rebalance clients); `h2_max_streams` — the
MAX_CONCURRENT_STREAMS advertised; `h2_initial_window` — the stream window advertised (request bodies larger
than it wait for the WINDOW_UPDATEs the server sends as it reads); `h2_small_conn_window` — the connection window
left at 65 535 and credited as DATA is read, so concurrent bodies also wait on the connection's window.
"""
from __future__ import annotations

import asyncio
import struct

from . import native as _native

PREFACE = b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n"

DATA, HEADERS, PRIORITY, RST_STREAM, SETTINGS, PUSH_PROMISE, PING, GOAWAY, WINDOW_UPDATE, CONTINUATION = range(10)
END_STREAM = ACK = 0x1
END_HEADERS = 0x4
PADDED = 0x8
PRIORITY_FLAG = 0x20

S_HEADER_TABLE_SIZE, S_ENABLE_PUSH, S_MAX_CONCURRENT_STREAMS, S_INITIAL_WINDOW_SIZE, S_MAX_FRAME_SIZE, \
    S_MAX_HEADER_LIST_SIZE = range(1, 7)
NO_ERROR, PROTOCOL_ERROR, INTERNAL_ERROR, FLOW_CONTROL_ERROR, _SETTINGS_TIMEOUT, STREAM_CLOSED, FRAME_SIZE_ERROR, \
    REFUSED_STREAM, CANCEL, COMPRESSION_ERROR = range(10)

OUR_WINDOW = 1 << 24  # per stream; the connection window is raised to 1 GiB at start
OUR_MAX_FRAME = 1 << 14

_HOP_BY_HOP = {"connection", "keep-alive", "transfer-encoding", "upgrade", "proxy-connection"}


def frame(ftype: int, flags: int, stream: int, payload: bytes = b"") -> bytes:
    n = len(payload)
    return struct.pack(">BHBBI", n >> 16, n & 0xFFFF, ftype, flags, stream & 0x7FFFFFFF) + payload


class _Stream:
    __slots__ = ("id", "send_window", "pending", "closed", "response_started", "eof_pending")

    def __init__(self, sid: int, window: int):
        self.id = sid
        self.send_window = window
        self.pending = bytearray()  # response DATA not yet within the windows
        self.eof_pending = False    # END_STREAM to send once `pending` is out
        self.closed = False         # reset, or our END_STREAM sent
        self.response_started = False


class H2Connection:
    """The HTTP/2 side of one `_ServerConn` (see the module doc).  Frames, stream assembly and HPACK are the
    extension's `H2ServerParser`; this class keeps the policy and the responses' flow control."""

    def __init__(self, conn, server):
        self.conn = conn
        self.server = server
        self.transport = conn.transport
        mod = _native.load(required=True)
        self.max_streams = int(server.h2_options.get("h2_max_streams", 0) or 0) or 250
        self.goaway_after = int(server.h2_options.get("h2_goaway_after", 0) or 0)
        # a small stream window makes a client's request bodies wait for our WINDOW_UPDATEs (tests)
        self.our_window = int(server.h2_options.get("h2_initial_window", 0) or 0) or OUR_WINDOW
        # the connection window left at the protocol's 65 535 (credited back as DATA is consumed): every client
        # request body then also waits for connection-level WINDOW_UPDATEs (tests)
        self.small_conn_window = bool(server.h2_options.get("h2_small_conn_window"))
        self.parser = mod.H2ServerParser(self.our_window < OUR_WINDOW or self.small_conn_window)
        self._encode = mod.h2_response
        self.streams: dict[int, _Stream] = {}  # dispatched, not yet answered to the end
        self.last_stream = 0
        self.served = 0
        self.goaway_sent = False
        self.conn_send_window = 65535
        self.peer_initial_window = 65535
        self.peer_max_frame = 16384
        self.recv_unacked = 0
        server.h2_stats["connections"] += 1
        # frames produced in one loop iteration (every response a batch of requests gets) leave in one write
        self._wbuf: list = []
        self._flush_scheduled = False
        # our SETTINGS, and the connection window raised to 1 GiB
        self._out(frame(SETTINGS, 0, 0, struct.pack(
            ">HIHIHIHI", S_MAX_CONCURRENT_STREAMS, self.max_streams, S_INITIAL_WINDOW_SIZE, self.our_window,
            S_MAX_FRAME_SIZE, OUR_MAX_FRAME, S_ENABLE_PUSH, 0)) +
            (b"" if self.small_conn_window else frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", (1 << 30) - 65535))))

    @property
    def open_streams(self) -> int:
        return len(self.streams)

    def _out(self, data: bytes) -> None:
        self._wbuf.append(data)
        if not self._flush_scheduled:
            self._flush_scheduled = True
            asyncio.get_running_loop().call_soon(self._flush_out)

    def _flush_out(self) -> None:
        self._flush_scheduled = False
        if self._wbuf and not self.conn.closed:
            data = b"".join(self._wbuf) if len(self._wbuf) > 1 else self._wbuf[0]
            self._wbuf.clear()
            self.transport.write(data)
        else:
            self._wbuf.clear()

    # ------------------------------------------------------------------ input
    def data_received(self, data: bytes) -> None:
        for ev in self.parser.feed(data):
            kind = ev[0]
            if kind == "req":
                self._request(*ev[1:])
            elif kind == "window":
                _, sid, inc = ev
                if sid == 0:
                    self.conn_send_window += inc
                    self._flush_all()
                else:
                    s = self.streams.get(sid)
                    if s is not None:
                        s.send_window += inc
                        self._flush(s)
            elif kind == "credit":  # DATA consumed: a stream's (small-window mode), or the connection's (sid 0)
                self._out(frame(WINDOW_UPDATE, 0, ev[1], struct.pack(">I", ev[2])))
                if self.small_conn_window and ev[1] != 0:
                    self._out(frame(WINDOW_UPDATE, 0, 0, struct.pack(">I", ev[2])))
            elif kind == "settings":
                for ident, value in ev[1]:
                    if ident == S_INITIAL_WINDOW_SIZE:
                        delta = value - self.peer_initial_window
                        self.peer_initial_window = value
                        for st in self.streams.values():
                            st.send_window += delta
                    elif ident == S_MAX_FRAME_SIZE:
                        self.peer_max_frame = value
                self._out(frame(SETTINGS, ACK, 0))
                self._flush_all()
            elif kind == "ping":
                self._out(frame(PING, ACK, 0, ev[1]))
            elif kind == "rst":
                st = self.streams.get(ev[1])
                if st is not None:
                    self._close(st)
            elif kind == "malformed":  # a pseudo-header after a regular field: Go's server resets the stream
                self.server.h2_stats["malformed"] += 1
                self._out(frame(RST_STREAM, 0, ev[1], struct.pack(">I", PROTOCOL_ERROR)))
            elif kind == "rst_closed":  # DATA on a stream that is not open
                self._out(frame(RST_STREAM, 0, ev[1], struct.pack(">I", STREAM_CLOSED)))
            elif kind == "goaway":
                self.goaway_sent = True  # the client is leaving: nothing new
            elif kind == "error":
                self._goaway(ev[1], ev[2])
                self._flush_out()
                self.transport.close()
                return

    def _request(self, sid: int, method: str, path: str, headers: dict, body: bytes) -> None:
        self.last_stream = max(self.last_stream, sid)
        if self.goaway_sent or len(self.streams) >= self.max_streams:
            self.server.h2_stats["refused"] += 1
            self._out(frame(RST_STREAM, 0, sid, struct.pack(">I", REFUSED_STREAM)))
            return
        s = self.streams[sid] = _Stream(sid, self.peer_initial_window)
        self._dispatch(s, method, path, headers, body)

    # ------------------------------------------------------------------ requests
    def _dispatch(self, s: _Stream, method: str, path: str, headers: dict, body: bytes) -> None:
        from .httpserver import Deferred, Request, Response
        req = Request(method, path, headers, body)
        req._conn = self.conn  # type: ignore[attr-defined]
        req._h2 = (self, s)    # type: ignore[attr-defined]
        self.served += 1
        st = self.server.h2_stats
        st["streams"] += 1
        if len(self.streams) > st["max_open"]:
            st["max_open"] = len(self.streams)
        if self.goaway_after and self.served >= self.goaway_after and not self.goaway_sent:
            self._goaway(NO_ERROR, "h2_goaway_after")
        fast = self.server.fast
        if fast is not None:
            try:
                resp = fast(req)
            except Exception as e:  # noqa: BLE001
                resp = Response(500, text=f"internal error: {e}")
            if isinstance(resp, Deferred):
                if resp.response is None:
                    resp.then(lambda r, s=s: self.respond(s, r))
                    return
                resp = resp.response
            if resp is not None:
                self.respond(s, resp)
                return
        task = asyncio.ensure_future(self.server.handler(req))
        task.add_done_callback(lambda t, s=s: self._done(s, t))

    def _done(self, s: _Stream, task: asyncio.Task) -> None:
        from .httpserver import Response
        try:
            resp = task.result()
        except Exception as e:  # noqa: BLE001
            resp = Response(500, text=f"internal error: {e}")
        if isinstance(resp, Response):
            self.respond(s, resp)
        elif not s.closed and not s.eof_pending:  # a stream handler returned without ending its body
            self.send_data(s, b"", end=True)

    def respond(self, s: _Stream, resp) -> None:
        if s.closed or self.conn.closed:
            return
        body = resp.body
        n = len(body)
        extra = [(k.lower(), str(v)) for k, v in resp.headers.items()] if resp.headers else []
        if n <= s.send_window and n <= self.conn_send_window and not s.pending:
            # the common case, whole within the windows: every frame of it encoded natively in one go
            self._out(self._encode(s.id, resp.status, resp.content_type, body, extra, self.peer_max_frame))
            s.send_window -= n
            self.conn_send_window -= n
            s.response_started = True
            self._close(s)
            return
        fields = [(":status", str(resp.status)), ("content-type", resp.content_type), ("content-length", str(n))]
        self.send_headers(s, fields + extra, end=not body)
        if body:
            self.send_data(s, body, end=True)

    def send_headers(self, s: _Stream, fields: list, end: bool = False) -> None:
        block = _native.load(required=True).hpack_encode(fields)
        s.response_started = True
        first, rest = block[:self.peer_max_frame], block[self.peer_max_frame:]
        flags = (END_STREAM if end else 0) | (0 if rest else END_HEADERS)
        out = [frame(HEADERS, flags, s.id, first)]
        while rest:
            chunk, rest = rest[:self.peer_max_frame], rest[self.peer_max_frame:]
            out.append(frame(CONTINUATION, 0 if rest else END_HEADERS, s.id, chunk))
        self._out(b"".join(out))
        if end:
            self._close(s)

    def send_data(self, s: _Stream, data: bytes, end: bool = False) -> None:
        if s.closed:
            return
        n = len(data)
        if not s.pending and n <= s.send_window and n <= self.conn_send_window and n <= self.peer_max_frame:
            # the common case (a watch event within the windows): one frame, no copy through `pending`
            s.send_window -= n
            self.conn_send_window -= n
            end = end or s.eof_pending
            self._out(frame(DATA, END_STREAM if end else 0, s.id, data))
            if end:
                s.eof_pending = False
                self._close(s)
            return
        s.pending += data
        s.eof_pending = s.eof_pending or end
        self._flush(s)

    def _flush(self, s: _Stream) -> None:
        out = []
        while s.pending and not s.closed:
            n = min(len(s.pending), s.send_window, self.conn_send_window, self.peer_max_frame)
            if n <= 0:
                break
            chunk = bytes(s.pending[:n])
            del s.pending[:n]
            s.send_window -= n
            self.conn_send_window -= n
            last = not s.pending and s.eof_pending
            out.append(frame(DATA, END_STREAM if last else 0, s.id, chunk))
            if last:
                s.eof_pending = False
                self._close(s)
        if not s.pending and s.eof_pending and not s.closed:  # an empty final frame
            out.append(frame(DATA, END_STREAM, s.id))
            s.eof_pending = False
            self._close(s)
        if out:
            self._out(b"".join(out))

    def _flush_all(self) -> None:
        for s in list(self.streams.values()):
            if s.pending or s.eof_pending:
                self._flush(s)

    def _close(self, s: _Stream) -> None:
        s.closed = True
        self.streams.pop(s.id, None)

    def _goaway(self, code: int, msg: str) -> None:
        if self.goaway_sent and code == NO_ERROR:
            return
        self.goaway_sent = True
        self.server.h2_stats["goaways"] += 1
        self._out(frame(GOAWAY, 0, 0, struct.pack(">II", self.last_stream, code) + msg.encode()[:64]))

    def connection_lost(self) -> None:
        for s in list(self.streams.values()):
            self._close(s)


class H2StreamWriter:
    """`StreamResponse` over HTTP/2 (a watch): the head as HEADERS, each write a DATA frame, EOF as END_STREAM."""

    def __init__(self, h2: H2Connection, s: _Stream):
        self.h2, self.s = h2, s

    def prepare(self, status: int, headers: dict) -> None:
        fields = [(":status", str(status))] + [(k.lower(), str(v)) for k, v in headers.items()
                                               if k.lower() not in _HOP_BY_HOP]
        self.h2.send_headers(self.s, fields)

    def write(self, data: bytes) -> None:
        if self.s.closed:
            raise ConnectionResetError("stream reset")
        self.h2.send_data(self.s, data)

    def write_eof(self) -> None:
        self.h2.send_data(self.s, b"", end=True)
