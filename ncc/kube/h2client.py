"""HTTP/2 for the Python clients: the coordinator's connection to the controller cluster (and the Python executor's
to its shards), as client-go's transport speaks it (`/root/reference/main.go:52-68` builds the clientsets; Go's
transport negotiates h2 by ALPN and multiplexes a clientset's requests on one connection).

`H2Pool` has `ConnectionPool`'s interface (`request`, `stream`, `close`), so `RestClient` uses either:

* every request is a stream; all streams opened in one loop iteration leave in one write (one TLS record), and
  a read brings many responses back at once — where HTTP/1.1 needs a connection per request in flight and a
  system call per request and per response;
* frames, HPACK and watch-body line splitting are native (`H2ClientParser`, `h2_request` in
  native/ncc_native.cpp over native/common/hpack.hpp); the policy is here: the server's stream limit (another
  connection opens only when every one is full), request-body flow control, GOAWAY (streams above its last id
  are retried on a fresh connection, as REFUSED_STREAM ones are), per-request deadlines, and the watch streams'
  windows, credited as their consumer takes the lines (the back-pressure `pause_reading` gives HTTP/1.1);
* negotiation: ALPN "h2" on TLS (`client-http2: auto`, the default), or prior knowledge on cleartext (`on`, for
  the shard clients: the controller cluster's negotiates, `ncc/config.py` `controller_http2`).
  A server that does not speak HTTP/2 — ALPN picks http/1.1, or it answers the preface with anything but
  SETTINGS — makes the pool fall back to HTTP/1.1 (`transport.ConnectionPool`) for good;
* error codes (the C++ executor's client does the same, native/executor/h2.hpp): a GOAWAY
  with an error code makes the re-sends of the streams it refused back off (50 ms doubling to 5 s) instead of
  going out at once; HTTP_1_1_REQUIRED in RST_STREAM or GOAWAY moves the pool to HTTP/1.1, with a warning; a
  WINDOW_UPDATE of 0 or one overflowing a window past 2^31-1 is a stream error on a stream (RST_STREAM) and a
  connection error on the connection; a connection error sends GOAWAY with its code before the close.
"""
from __future__ import annotations

import asyncio
import os
import ssl as _ssl
import struct
from collections import deque
from urllib.parse import urlsplit

from .. import native as _native
from ..aio import wait_timeout
from . import errors as E
from .transport import ConnectionPool, _Response

_mod = _native.load()
_Parser = getattr(_mod, "H2ClientParser", None) if _mod is not None else None
_h2_request = getattr(_mod, "h2_request", None) if _mod is not None else None
_hpack_encode = getattr(_mod, "hpack_encode", None) if _mod is not None else None

AVAILABLE = _Parser is not None
_BODY_METHODS = frozenset(("POST", "PUT", "PATCH"))
_NO_BODY = b""
# RFC 9113 error codes used here
NO_ERROR, PROTOCOL_ERROR, FLOW_CONTROL_ERROR, CANCEL, REFUSED_STREAM = 0x0, 0x1, 0x3, 0x8, 0x7
ENHANCE_YOUR_CALM, HTTP_1_1_REQUIRED = 0xb, 0xd
MAX_WINDOW = 0x7FFFFFFF  # a flow-control window never exceeds 2^31-1 (RFC 9113 §6.9.1)
WATCH_CREDIT = 1 << 16  # a watch stream's consumed bytes are credited back in updates of at least this much


def _frame(type_: int, flags: int, sid: int, payload: bytes) -> bytes:
    return struct.pack(">I", len(payload))[1:] + struct.pack(">BBI", type_, flags, sid & 0x7fffffff) + payload


def _window_update(sid: int, n: int) -> bytes:
    return _frame(8, 0, sid, struct.pack(">I", n & 0x7fffffff))


def _tap(tap, lines: list) -> None:
    try:
        tap(lines)
    except Exception:  # noqa: BLE001 — a tap must not break the stream its consumer reads
        import logging
        logging.getLogger("ncc.transport").exception("watch line tap failed")


class _NoH2(Exception):
    """The server does not speak HTTP/2 on this connection."""


class _Retry(Exception):
    """The server did not process the stream (REFUSED_STREAM, or above a GOAWAY's last id): safe to send again.
    `refused`: REFUSED_STREAM — the same server is busy, so the retry backs off (a GOAWAY's goes straight to a
    new connection)."""

    def __init__(self, refused: bool = False):
        super().__init__()
        self.refused = refused


MAX_STREAM_ID = 0x7FFFFFF0  # a connection's client stream ids run out below 2^31 (RFC 9113 §5.1.1)
MAX_UNPROCESSED_RETRIES = 16  # re-sends of a request no server processed (a GOAWAY each time is progress elsewhere)


class _Stream:
    __slots__ = ("sid", "fut", "deadline", "what", "body", "send_window", "watch", "lines", "event", "done",
                 "tap", "uncredited", "head")

    def __init__(self, sid: int, fut, what: str, send_window: int, watch: bool = False):
        self.sid, self.fut, self.what, self.send_window, self.watch = sid, fut, what, send_window, watch
        self.deadline = None
        self.body = _NO_BODY  # request body still to send (blocked on a flow-control window)
        self.lines: deque | None = deque() if watch else None
        self.event: asyncio.Event | None = asyncio.Event() if watch else None
        self.done = False
        self.tap = None
        self.uncredited = 0
        self.head = None


class _H2Conn(asyncio.Protocol):
    """One HTTP/2 connection: its streams, send windows and the native parser of what the server sends."""

    def __init__(self, pool: "H2Pool"):
        self.pool = pool
        self.parser = _Parser()
        self.transport: asyncio.Transport | None = None
        self.streams: dict[int, _Stream] = {}
        self.next_sid = 1
        self.peer_max_streams = 100  # until the server's SETTINGS say otherwise
        # streams this connection may carry: the server's limit, lowered for good to 7/8 of what was in flight each
        # time the server refuses a stream (REFUSED_STREAM / ENHANCE_YOUR_CALM) — a server whose own count of open
        # streams lags ours (nghttp2 under Node frees a stream some time after its END_STREAM went out) refuses
        # streams opened at or near its limit
        self.stream_cap = pool.stream_cap
        self.peer_window = 65535     # its SETTINGS_INITIAL_WINDOW_SIZE: each new stream's send window
        self.peer_max_frame = 16384
        self.send_window = 65535     # the connection's
        self.blocked: deque = deque()
        self.ready = asyncio.get_running_loop().create_future()
        self.last_recv = asyncio.get_running_loop().time()
        self.ping_sent = 0.0         # loop time of an unanswered PING (liveness check), 0 = none
        self.draining = False        # GOAWAY received (or sent): no new streams
        self.lost_why = "closed by peer"
        self.closed = False
        self._out: list = []
        self._flush_handle = None

    # ------------------------------------------------------------------ protocol
    def connection_made(self, transport):
        self.transport = transport
        if self.pool.tls:
            sslobj = transport.get_extra_info("ssl_object")
            if sslobj is None or sslobj.selected_alpn_protocol() != "h2":
                self._fail_ready(_NoH2("the server did not negotiate HTTP/2 (ALPN)"))
                self.closed = True
                transport.close()
                return
        transport.write(_Parser.preface())

    def _fail_ready(self, exc: BaseException) -> None:
        if not self.ready.done():
            self.ready.set_exception(exc)
            self.ready.exception()  # retrieved: a pool that gave up on the connect must not log it

    def connection_lost(self, exc):
        self.closed = True
        if self._flush_handle is not None:
            self._flush_handle.cancel()
            self._flush_handle = None
        if not self.ready.done():
            # closed before its SETTINGS: on cleartext with prior knowledge, an HTTP/1.1 server hanging up on the
            # preface; on TLS (ALPN said h2) a plain failure
            self._fail_ready(_NoH2("closed before SETTINGS") if not self.pool.tls else
                             E.TransportError(f"connection lost: {exc or 'closed by peer'}"))
        err = E.TransportError(f"connection lost: {exc or self.lost_why}")
        for st in list(self.streams.values()):
            self._end(st, err)
        self.streams.clear()
        self.blocked.clear()
        self.pool._discard(self)

    def pause_writing(self):  # pragma: no cover - large request bodies only
        pass

    def resume_writing(self):  # pragma: no cover
        pass

    def data_received(self, data: bytes):
        self.last_recv = self.pool._now()
        events, out = self.parser.feed(data)
        if out:
            self._send(out)
        streams = self.streams
        for ev in events:
            kind = ev[0]
            if kind == "resp":
                st = streams.pop(ev[1], None)
                if st is not None:
                    if not st.fut.done():
                        st.fut.set_result(_Response(ev[2], _NO_HEADERS if ev[3] is None else {"retry-after": ev[3]},
                                                    ev[4]))
                    self.pool._stream_closed(self)
            elif kind == "lines":
                st = streams.get(ev[1])
                if st is None:
                    continue
                lines = ev[2]
                if lines:
                    if st.tap is not None:
                        _tap(st.tap, lines)
                    st.lines.extend(lines)
                if st.tap is not None:
                    if ev[3]:
                        self._send(_window_update(st.sid, ev[3]))  # a tapped stream is read as it arrives
                else:
                    st.uncredited += ev[3]
                if ev[4]:
                    st.done = True
                    del streams[st.sid]
                    self.pool._stream_closed(self)
                st.event.set()
            elif kind == "head":
                st = streams.get(ev[1])
                if st is not None and not st.fut.done():
                    st.head = _Response(ev[2], _NO_HEADERS if ev[3] is None else {"retry-after": ev[3]}, b"")
                    st.fut.set_result(st.head)
            elif kind == "settings":
                if not self._settings(ev[1]):
                    return
            elif kind == "window":
                if not self._window(ev[1], ev[2]):
                    return
            elif kind == "rst":
                st = streams.pop(ev[1], None)
                code = ev[2]
                if st is not None:
                    # REFUSED_STREAM: not processed; HTTP_1_1_REQUIRED: refused for the protocol — both safe to send
                    # again (the second over HTTP/1.1, from now on); ENHANCE_YOUR_CALM: the server sheds load
                    # (nghttp2 under Node resets the streams it will not take with it) — again after a backoff
                    if code == ENHANCE_YOUR_CALM:
                        self.pool.stats["h2_calm"] += 1
                        self.pool._back_off(False, "RST_STREAM ENHANCE_YOUR_CALM")
                    if code in (REFUSED_STREAM, ENHANCE_YOUR_CALM):  # 7/8 of what was in flight, for good
                        n = min(self.stream_cap, len(streams) + 1)
                        self.stream_cap = max(1, n - max(1, n // 8))
                        self.pool.stream_cap = min(self.pool.stream_cap, self.stream_cap)  # and the next connections
                    self._end(st, _Retry(code == REFUSED_STREAM)
                              if code in (REFUSED_STREAM, HTTP_1_1_REQUIRED, ENHANCE_YOUR_CALM) else
                              E.TransportError(f"{st.what}: stream reset by the server (code {code})"))
                    if code == REFUSED_STREAM:
                        self.pool.stats["h2_refused"] += 1
                    self.pool._stream_closed(self)
                if code == HTTP_1_1_REQUIRED:
                    self.draining = True
                    self.pool._downgrade("RST_STREAM HTTP_1_1_REQUIRED")
            elif kind == "goaway":
                self._goaway(ev[1], ev[2])
            elif kind == "noh2":
                self._fail_ready(_NoH2("the server answered the HTTP/2 preface with something else"))
                self.close()
                return
            elif kind == "error":
                self._connection_error(ev[1], ev[2])
                return
        if self.draining and not streams and not self.closed:
            self.close()  # after a GOAWAY, once the streams it let finish have finished

    def _connection_error(self, code: int, why: str) -> None:
        """RFC 9113 §5.4.1: GOAWAY with the error code, then close; every stream fails."""
        self._send(_frame(7, 0, 0, struct.pack(">II", 0, code) + why.encode()[:200]))
        self._flush()
        err = E.TransportError(f"HTTP/2 connection error: {why}")
        self._fail_ready(err)
        for st in list(self.streams.values()):
            self._end(st, err)
        self.streams.clear()
        self.close()

    # ------------------------------------------------------------------ frames in
    def _settings(self, kv) -> bool:
        for k, v in kv:
            if k == 0x3:
                self.peer_max_streams = v
            elif k == 0x4:
                if v > MAX_WINDOW:
                    self._connection_error(FLOW_CONTROL_ERROR, "INITIAL_WINDOW_SIZE above 2^31-1")
                    return False
                delta = v - self.peer_window
                self.peer_window = v
                for st in self.streams.values():
                    st.send_window += delta
                    if st.send_window > MAX_WINDOW:  # §6.9.2: a connection error
                        self._connection_error(FLOW_CONTROL_ERROR, "INITIAL_WINDOW_SIZE overflows a stream window")
                        return False
            elif k == 0x5:
                self.peer_max_frame = v
        if not self.ready.done():
            self.ready.set_result(None)
        self._drain_blocked()
        self.pool._stream_closed(self)  # a raised stream limit is room for waiters
        return True

    def _window(self, sid: int, n: int) -> bool:
        """WINDOW_UPDATE (§6.9): an increment of 0, or a window pushed past 2^31-1, is a connection error on
        the connection and a stream error (RST_STREAM, the stream fails) on a stream.  False: the connection
        is gone."""
        if sid == 0:
            if n == 0:
                self._connection_error(PROTOCOL_ERROR, "WINDOW_UPDATE of 0 on the connection")
                return False
            if self.send_window + n > MAX_WINDOW:
                self._connection_error(FLOW_CONTROL_ERROR, "connection window past 2^31-1")
                return False
            self.send_window += n
        else:
            st = self.streams.get(sid)
            if st is None:
                return True
            bad = PROTOCOL_ERROR if n == 0 else FLOW_CONTROL_ERROR if st.send_window + n > MAX_WINDOW else 0
            if bad:
                self.streams.pop(sid, None)
                self.parser.forget(sid)
                self._send(_frame(3, 0, sid, struct.pack(">I", bad)))
                self._end(st, E.TransportError(f"{st.what}: HTTP/2 stream error: " +
                                               ("WINDOW_UPDATE of 0" if n == 0 else "stream window past 2^31-1")))
                self.pool._stream_closed(self)
                return True
            st.send_window += n
        self._drain_blocked()
        return True

    def _goaway(self, last: int, code: int) -> None:
        self.draining = True
        self.pool.stats["h2_goaways"] += 1
        if code == HTTP_1_1_REQUIRED:
            self.pool._downgrade("GOAWAY HTTP_1_1_REQUIRED")
        elif code != NO_ERROR:
            self.pool._goaway_error(code)
        for sid in [s for s in self.streams if s > last]:
            st = self.streams.pop(sid)
            self._end(st, _Retry())
        if not self.streams:
            self.close()
        self.pool._stream_closed(self)

    def _end(self, st: _Stream, exc: BaseException) -> None:
        if st.watch:
            st.done = True
            if not st.fut.done():
                st.fut.set_exception(exc if not isinstance(exc, _Retry) else
                                     E.TransportError(f"{st.what}: refused by the server"))
            st.event.set()
        elif not st.fut.done():
            st.fut.set_exception(exc)

    # ------------------------------------------------------------------ frames out
    def _send(self, data: bytes) -> None:
        self._out.append(data)
        if self._flush_handle is None:
            self._flush_handle = asyncio.get_running_loop().call_soon(self._flush)

    def _flush(self) -> None:
        self._flush_handle = None
        out, self._out = self._out, []
        if out and not self.closed and self.transport is not None:
            self.transport.write(out[0] if len(out) == 1 else b"".join(out))

    def has_room(self) -> bool:
        return not self.closed and not self.draining and len(self.streams) < min(self.peer_max_streams, self.stream_cap)

    def open(self, method: str, target: str, fixed: bytes, clen: int, body: bytes, what: str,
             watch: bool = False) -> _Stream:
        sid = self.next_sid
        self.next_sid += 2
        if self.next_sid >= MAX_STREAM_ID:
            self.draining = True  # stream ids spent (2^31): no new streams here; closed once these finish
        fut = asyncio.get_running_loop().create_future()
        st = _Stream(sid, fut, what, self.peer_window, watch)
        self.streams[sid] = st
        if watch:
            self.parser.watch(sid)
        n = len(body)
        if n <= st.send_window and n <= self.send_window:
            data = _h2_request(sid, method, target, fixed, clen, body, True, self.peer_max_frame)
            if len(self.streams) == 1 and not self._out and self.transport is not None:
                # the only stream in flight: out now (batching would cost it a loop iteration and gain nothing)
                self.transport.write(data)
            else:
                self._send(data)
            st.send_window -= n
            self.send_window -= n
        else:  # the body waits for WINDOW_UPDATEs
            self._send(_h2_request(sid, method, target, fixed, clen, _NO_BODY, False, self.peer_max_frame))
            st.body = body
            self.blocked.append(st)
            self._drain_blocked()
        self.pool.stats["h2_streams"] += 1
        self.pool._arm_sweep()
        return st

    def _drain_blocked(self) -> None:
        while self.blocked and self.send_window > 0:
            st = self.blocked[0]
            if st.done or self.streams.get(st.sid) is not st:
                self.blocked.popleft()
                continue
            room = min(st.send_window, self.send_window)
            if room <= 0:
                # this stream waits for its own window; others behind it may not
                self.blocked.rotate(-1)
                if all(s.send_window <= 0 for s in self.blocked):
                    return
                continue
            n = min(room, len(st.body), self.peer_max_frame)
            chunk, st.body = st.body[:n], st.body[n:]
            st.send_window -= n
            self.send_window -= n
            last = not st.body
            self._send(_frame(0, 0x1 if last else 0, st.sid, chunk))
            if last:
                self.blocked.popleft()

    def cancel(self, st: _Stream) -> None:
        """Reset a stream the client gives up on (a deadline, a closed watch)."""
        if self.streams.pop(st.sid, None) is not None:
            self.parser.forget(st.sid)
            self._send(_frame(3, 0, st.sid, struct.pack(">I", CANCEL)))
            self.pool._stream_closed(self)

    def ping(self, now: float) -> None:
        self.ping_sent = now
        self._send(_frame(6, 0, 0, b"ncc-live"))

    def credit(self, st: _Stream) -> None:
        if st.uncredited >= WATCH_CREDIT and not st.done:
            self._send(_window_update(st.sid, st.uncredited))
            st.uncredited = 0

    def close(self) -> None:
        if not self.closed:
            self.closed = True
            if self.transport is not None:
                if self._out:
                    self._flush()
                self.transport.close()

    def abort(self, why: str) -> None:
        """Drop a dead connection at once (close() would wait for its send buffer to drain)."""
        self.lost_why = why
        self.closed = True
        if self.transport is not None:
            self.transport.abort()


_NO_HEADERS: dict = {}


class H2Pool:
    """HTTP/2 connections to one apiserver, `ConnectionPool`'s interface.  `prior_knowledge`: speak HTTP/2 on
    cleartext without negotiation (TLS always negotiates by ALPN)."""

    SWEEP_PERIOD = 0.5

    def __init__(self, server: str, *, ssl_context: _ssl.SSLContext | None = None, server_hostname: str | None = None,
                 max_size: int = 64, connect_timeout: float = 10.0, pipeline_depth: int = 1,
                 prior_knowledge: bool = False, proxy: str | None = None,
                 fallback_ssl_context: _ssl.SSLContext | None = None):
        """`fallback_ssl_context`: the TLS context of the HTTP/1.1 fallback pool — one that offers only
        "http/1.1" by ALPN (`ssl_context` offers "h2" too, and a server behind a mixed load balancer that picks
        h2 would then be spoken to in HTTP/1.1 over an h2 connection)."""
        if not AVAILABLE:
            raise RuntimeError("HTTP/2 needs the native extension (ncc/_native)")
        u = urlsplit(server)
        self.server = server
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.authority = u.netloc
        self.tls = u.scheme == "https"
        self.ssl = ssl_context if self.tls else None
        if self.ssl is not None:
            self.ssl.set_alpn_protocols(["h2", "http/1.1"])
        self.fallback_ssl = fallback_ssl_context if self.tls else None
        if self.fallback_ssl is not None:
            self.fallback_ssl.set_alpn_protocols(["http/1.1"])
        self.server_hostname = server_hostname
        self.max_size = max(1, max_size)
        self.connect_timeout = connect_timeout
        self.pipeline_depth = pipeline_depth
        self.prior_knowledge = prior_knowledge
        self.proxy = proxy  # an HTTP CONNECT proxy (ncc/kube/proxy.py); HTTP/2 runs inside the tunnel
        self.conns: list[_H2Conn] = []
        self._connecting: asyncio.Future | None = None
        self._waiters: deque = deque()
        self._fixed: dict = {}
        self._sweep_handle = None
        self.fallback: ConnectionPool | None = None
        self.opened = 0
        # liveness, as client-go's transport: a connection with streams open that read nothing for READ_IDLE
        # seconds (or whose stream just timed out) is PINGed, and closed when PING_TIMEOUT passes without an
        # answer — a silently dead TCP connection would otherwise hold every stream until the kernel gives up
        self.read_idle = float(os.environ.get("HTTP2_READ_IDLE_TIMEOUT_SECONDS", "30") or 30)
        self.ping_timeout = float(os.environ.get("HTTP2_PING_TIMEOUT_SECONDS", "15") or 15)
        self.stats = {"h2_streams": 0, "h2_refused": 0, "h2_goaways": 0, "h2_dead": 0, "h2_goaway_errors": 0,
                      "h2_downgraded": 0, "h2_calm": 0}
        self.backoff_until = 0.0  # after a GOAWAY with an error code: refused streams re-send from then on
        self._backoff_n = 0       # error GOAWAYs in a row (the backoff doubles with each; a response resets it)
        self.stream_cap = 1 << 31  # the lowest per-connection stream cap a refusal taught (_H2Conn.stream_cap)

    @property
    def protocol(self) -> str:
        return "http/1.1" if self.fallback is not None else "h2"

    # ------------------------------------------------------------------ connections
    async def _connect(self) -> _H2Conn:
        loop = asyncio.get_running_loop()
        kw = {}
        if self.ssl is not None:
            kw["ssl"] = self.ssl
            kw["server_hostname"] = self.server_hostname or self.host
        try:
            if self.proxy:
                from .proxy import open_tunnel
                sock = await open_tunnel(self.proxy, self.host, self.port, self.connect_timeout)
                coro = loop.create_connection(lambda: _H2Conn(self), sock=sock, **kw)
            else:
                coro = loop.create_connection(lambda: _H2Conn(self), self.host, self.port, **kw)
            _, conn = await wait_timeout(coro, self.connect_timeout)
        except (OSError, asyncio.TimeoutError, _ssl.SSLError) as e:
            raise E.TransportError(f"connect {self.host}:{self.port}: {type(e).__name__}: {e}") from e
        try:
            await wait_timeout(asyncio.shield(conn.ready), self.connect_timeout)
        except asyncio.TimeoutError as e:
            conn.close()
            raise (_NoH2("no SETTINGS from the server") if not self.tls else
                   E.TransportError(f"connect {self.host}:{self.port}: no HTTP/2 SETTINGS")) from e
        self.opened += 1
        self.conns.append(conn)
        return conn

    def _downgrade(self, why: str) -> None:
        """HTTP_1_1_REQUIRED: every request from now on over HTTP/1.1, as when ALPN refuses h2; the HTTP/2
        connections finish the streams they have and take no new ones."""
        if self.fallback is not None:
            return
        import logging
        logging.getLogger("ncc.transport").warning(
            "%s from %s:%s: the server requires HTTP/1.1; using HTTP/1.1 for it from now on", why, self.host, self.port)
        self.stats["h2_downgraded"] = 1
        for c in self.conns:
            c.draining = True
        self._h1()

    def _goaway_error(self, code: int) -> None:
        """A GOAWAY with an error code (ENHANCE_YOUR_CALM: we are being shed; or a server-side error): the streams
        it refused wait before they are sent again (`_back_off`)."""
        self.stats["h2_goaway_errors"] += 1
        self._back_off(True, f"GOAWAY with HTTP/2 error {code:#x}")

    def _back_off(self, loud: bool, why: str) -> None:
        """Refused streams re-send from `backoff_until` on: 50 ms, doubling with every refusal in a row up to 5 s (a
        response resets it).  `loud`: a warning each time (a GOAWAY); a stream reset only at the start of a run."""
        wait = min(5.0, 0.05 * (2 ** min(self._backoff_n, 7)))
        if loud or self._backoff_n == 0:
            import logging
            logging.getLogger("ncc.transport").warning("%s from %s:%s; re-sending the refused streams after %d ms",
                                                       why, self.host, self.port, int(wait * 1000))
        self._backoff_n += 1
        self.backoff_until = max(self.backoff_until, self._now() + wait)

    def _h1(self) -> ConnectionPool:
        if self.fallback is None:
            ctx = self.fallback_ssl if self.fallback_ssl is not None else self.ssl
            self.fallback = ConnectionPool(self.server, ssl_context=ctx, server_hostname=self.server_hostname,
                                           max_size=self.max_size, connect_timeout=self.connect_timeout,
                                           pipeline_depth=self.pipeline_depth, proxy=self.proxy)
        return self.fallback

    def _pick(self) -> _H2Conn | None:
        for c in self.conns:
            if c.has_room():
                return c
        return None

    async def _conn(self) -> _H2Conn | None:
        """A connection with room for a stream; None once the server turned out not to speak HTTP/2."""
        while True:
            c = self._pick()
            if c is not None:
                return c
            if self.fallback is not None:
                return None
            if self._connecting is not None:
                await asyncio.shield(self._connecting)  # one connect at a time; then look again
                continue
            if len([c for c in self.conns if not c.closed]) < self.max_size:
                fut = self._connecting = asyncio.get_running_loop().create_future()
                try:
                    return await self._connect()
                except _NoH2 as e:
                    if self.opened:
                        # it spoke HTTP/2 before (a load balancer whose backends differ, a server downgraded):
                        # fall back as on the first connection, as Go's transport decides per connection
                        import logging
                        logging.getLogger("ncc.transport").warning(
                            "%s:%s no longer offers HTTP/2 (%s); using HTTP/1.1 for it", self.host, self.port, e)
                    self._h1()  # from now on, every request goes there
                    return None
                finally:
                    self._connecting = None
                    fut.set_result(None)
            w = asyncio.get_running_loop().create_future()
            self._waiters.append(w)
            await w

    def _stream_closed(self, c: _H2Conn) -> None:
        """Room on `c` (or `c` gone): wake as many waiters as it has free streams; they pick again."""
        if not self._waiters:
            return
        free = min(c.peer_max_streams, c.stream_cap) - len(c.streams) if c.has_room() else \
            (1 if c.closed or c.draining else 0)
        while self._waiters and free > 0:
            w = self._waiters.popleft()
            if not w.done():
                w.set_result(None)
                free -= 1

    def _discard(self, c: _H2Conn) -> None:
        try:
            self.conns.remove(c)
        except ValueError:
            pass
        while self._waiters:  # let them connect afresh
            w = self._waiters.popleft()
            if not w.done():
                w.set_result(None)

    def _fixed_block(self, headers: dict, block: bytes | None) -> bytes:
        key = block if block is not None else tuple(headers.items())
        got = self._fixed.get(key)
        if got is None:
            if len(self._fixed) > 16:
                self._fixed.clear()
            fields = [(":scheme", "https" if self.tls else "http"), (":authority", headers.get("Host", self.authority))]
            fields += [(k.lower(), str(v)) for k, v in headers.items() if k.lower() not in ("host", "connection")]
            got = self._fixed[key] = _hpack_encode(fields)
        return got

    # ------------------------------------------------------------------ deadlines
    def _arm_sweep(self) -> None:
        if self._sweep_handle is None:
            self._sweep_handle = asyncio.get_running_loop().call_later(self.SWEEP_PERIOD, self._sweep)

    @staticmethod
    def _now() -> float:
        return asyncio.get_running_loop().time()

    def _sweep(self) -> None:
        """Every SWEEP_PERIOD while streams are open: request deadlines and connection liveness."""
        self._sweep_handle = None
        now = self._now()
        pending = False
        for c in list(self.conns):
            late = False
            for st in [s for s in c.streams.values() if s.deadline is not None and s.deadline <= now]:
                c.cancel(st)
                c._end(st, E.TransportError(f"{st.what}: timed out"))
                late = True
            if c.ping_sent and c.last_recv >= c.ping_sent:
                c.ping_sent = 0.0  # anything read since the PING answers it
            if c.ping_sent and now - c.ping_sent >= self.ping_timeout:
                self.stats["h2_dead"] += 1
                import logging
                logging.getLogger("ncc.transport").warning(
                    "HTTP/2 connection to %s:%s: no answer to PING within %.0f s; closing it", self.host, self.port,
                    self.ping_timeout)
                c.abort("no answer to PING")  # its streams fail; requests and watches start over on a new one
                continue
            if c.streams:
                pending = True
                if not c.ping_sent and (late or now - c.last_recv >= self.read_idle):
                    c.ping(now)
        if pending:
            self._arm_sweep()

    # ------------------------------------------------------------------ API
    async def request(self, method: str, target: str, headers: dict, body: bytes | None,
                      timeout: float | None = 30.0, block: bytes | None = None) -> _Response:
        if self.fallback is not None:
            return await self.fallback.request(method, target, headers, body, timeout=timeout, block=block)
        fixed = self._fixed_block(headers, block)
        clen = len(body) if body is not None else (0 if method in _BODY_METHODS else -1)
        what = f"{method} {target}"
        for attempt in range(MAX_UNPROCESSED_RETRIES + 1):
            c = self._pick() if self.fallback is None else None
            if c is None:
                c = await self._conn()
            if c is None:
                return await self.fallback.request(method, target, headers, body, timeout=timeout, block=block)
            st = c.open(method, target, fixed, clen, body or _NO_BODY, what)
            if timeout:
                st.deadline = asyncio.get_running_loop().time() + timeout
                self._arm_sweep()
            try:
                resp = await st.fut
                self._backoff_n = 0
                return resp
            except _Retry as r:
                if attempt < MAX_UNPROCESSED_RETRIES:
                    wait = self.backoff_until - self._now()
                    if r.refused:
                        wait = max(wait, min(0.001 * (2 ** attempt), 0.1))
                    if wait > 0:
                        await asyncio.sleep(wait)
                    continue
                raise E.TransportError(f"{what}: refused by the server") from None
            except asyncio.CancelledError:
                c.cancel(st)
                raise
        raise E.TransportError("unreachable")  # pragma: no cover

    async def stream(self, target: str, headers: dict, timeout: float | None = None, batch: bool = False,
                     on_lines=None):
        """`ConnectionPool.stream` over a stream of a shared connection: yields (response, None) — or (response,
        error body) for a non-2xx — then (None, line) or, with `batch`, (None, [lines])."""
        if self.fallback is None:
            c = self._pick() or await self._conn()
        else:
            c = None
        if c is None:
            async for x in self.fallback.stream(target, headers, timeout=timeout, batch=batch, on_lines=on_lines):
                yield x
            return
        loop = asyncio.get_running_loop()
        st = c.open("GET", target, self._fixed_block(headers, None), -1, _NO_BODY, f"GET {target}", watch=True)
        st.deadline = loop.time() + self.connect_timeout + 20  # for the response head
        self._arm_sweep()
        stream_timer = None
        try:
            resp = await st.fut
            st.deadline = None
            if timeout:
                stream_timer = loop.call_later(timeout, self._end_watch, c, st)
            if resp.status >= 300:
                while not st.done:
                    st.event.clear()
                    await st.event.wait()
                yield resp, b"\n".join(st.lines)
                return
            if on_lines is not None:
                if st.lines:
                    on_lines(list(st.lines))
                st.tap = on_lines
                if st.uncredited:
                    c._send(_window_update(st.sid, st.uncredited))
                    st.uncredited = 0
            yield resp, None
            while True:
                if batch:
                    while st.lines:
                        lines = list(st.lines)
                        st.lines.clear()
                        c.credit(st)
                        yield None, lines
                else:
                    while st.lines:
                        yield None, st.lines.popleft()
                        c.credit(st)
                if st.done:
                    return
                st.event.clear()
                await st.event.wait()
        finally:
            if stream_timer is not None:
                stream_timer.cancel()
            if not st.done:
                c.cancel(st)
                st.done = True

    @staticmethod
    def _end_watch(c: _H2Conn, st: _Stream) -> None:
        if not st.done:
            c.cancel(st)
            st.done = True
            st.event.set()

    def close(self) -> None:
        if self._sweep_handle is not None:
            self._sweep_handle.cancel()
            self._sweep_handle = None
        for c in list(self.conns):
            c.close()
        self.conns.clear()
        if self.fallback is not None:
            self.fallback.close()
