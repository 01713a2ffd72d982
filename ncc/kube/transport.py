"""Lean HTTP/1.1 keep-alive transport on raw asyncio Protocols.

A generic HTTP client (aiohttp) spends ~100-150 µs of Python per request on URL objects,
multidict headers, tracing hooks and timers.  A controller that fans every change out to N
clusters is bound by exactly that per-request cost, so the default transport speaks the small
subset of HTTP/1.1 a kube-apiserver needs directly on asyncio transports:

* keep-alive connections from a bounded pool; with `pipeline_depth > 1`, once every connection is
  busy further requests are pipelined (HTTP/1.1) onto the least-loaded one, and all requests queued on
  a connection within one loop iteration go out in a single write;
* pre-encoded request heads, `Content-Length` bodies;
* response framing by `Content-Length` or `Transfer-Encoding: chunked`, incremental parsing
  in `data_received` (no per-byte Python loops);
* streaming mode for watches: chunked frames are decoded and split into JSON lines as they
  arrive, with back-pressure (`pause_reading`) when the consumer falls behind.

`AiohttpTransport` keeps the aiohttp path available (`transport: aiohttp`).
"""
from __future__ import annotations

import asyncio
import ssl as _ssl
from collections import deque
from urllib.parse import urlsplit

from .. import native as _native
from ..aio import wait_timeout
from . import errors as E

_CRLF2 = b"\r\n\r\n"


_native_mod = _native.load()
_parse_native = getattr(_native_mod, "parse_response_head", None) if _native_mod is not None else None
_chunk_lines = getattr(_native_mod, "chunk_lines", None) if _native_mod is not None else None
_NO_HEADERS: dict = {}


def _parse_head_py(head: bytes) -> tuple:
    """(status, content_length | -1, chunked, connection_close, headers) — the pure-Python fallback."""
    lines = head.split(b"\r\n")
    parts = lines[0].split(b" ", 2)
    try:
        status = int(parts[1])
    except (IndexError, ValueError) as e:
        raise E.TransportError(f"malformed response head: {lines[0][:80]!r}") from e
    h = {}
    for ln in lines[1:]:
        k, _, v = ln.partition(b":")
        h[k.strip().lower().decode("latin-1")] = v.strip().decode("latin-1")
    clen = int(h["content-length"]) if "content-length" in h else -1
    return (status, clen, "chunked" in h.get("transfer-encoding", "").lower(),
            h.get("connection", "").lower() == "close", h)


class _Response:
    __slots__ = ("status", "headers", "body")

    def __init__(self, status: int, headers: dict, body: bytes):
        self.status, self.headers, self.body = status, headers, body


class _Conn(asyncio.Protocol):
    """One HTTP/1.1 connection.  Requests are answered in order (`pending` futures, FIFO); a streaming
    (watch) connection carries exactly one exchange."""

    HIGH_WATER = 64
    # a tapped stream (the watch relay's) keeps reading while its consumer works through a burst: the tap
    # must see lines as they arrive, so the buffer may hold a whole wave (lines are ~1 KB)
    TAPPED_HIGH_WATER = 1 << 16

    def __init__(self, pool: "ConnectionPool"):
        self.pool = pool
        self.transport: asyncio.Transport | None = None
        self.buf = bytearray()
        self.closed = False
        self.uses = 0
        self.pending: deque = deque()
        self._out: list = []
        self._flush_handle = None
        self.stream: deque | None = None
        # streams: callable(lines) seeing every complete line as it arrives, before the consumer does (the
        # coordinator's watch relay forwards lines from here, whatever its informer is busy with)
        self.line_tap = None
        self.deadline: float | None = None  # loop time by which the in-flight exchange must complete
        self.deadline_what = ""
        self.timed_out = False
        self._reset()

    @property
    def fut(self) -> asyncio.Future | None:
        return self.pending[0] if self.pending else None

    def _reset(self):
        self.head_done = False
        self.status = 0
        self.headers: dict = {}
        self.clen = -1
        self.chunked = False
        self.until_close = False
        self.body = bytearray()
        self.chunk_left = -1  # bytes left in current chunk (-1: expecting size line)
        self.stream_event: asyncio.Event | None = None
        self.stream_done = False
        self.linebuf = bytearray()
        self.paused = False
        self.keep_alive = True

    # ---------------------------------------------------------------- protocol
    def connection_made(self, transport):
        self.transport = transport

    def connection_lost(self, exc):
        self.closed = True
        fut = self.fut
        if fut is not None and not fut.done() and self.until_close and self.head_done:
            self.pending.popleft()
            fut.set_result(_Response(self.status, self.headers, bytes(self.body)))
        while self.pending:
            f = self.pending.popleft()
            if not f.done():
                f.set_exception(E.TransportError(f"connection lost: {exc or 'closed by peer'}"))
        if self.stream is not None:
            self.stream_done = True
            if self.stream_event is not None:
                self.stream_event.set()
        self.pool._discard(self)

    def pause_writing(self):  # pragma: no cover - large request bodies only
        pass

    def resume_writing(self):  # pragma: no cover
        pass

    def data_received(self, data: bytes):
        if not self.buf and not self.head_done and self.stream is None and self.pending:
            # fast path: a whole API response in one read (the common case) is framed straight from `data`
            i = data.find(_CRLF2)
            if i >= 0:
                self._parse_head(data[:i])
                if self.head_done and not self.chunked and 0 <= self.clen <= len(data) - i - 4:
                    end = i + 4 + self.clen
                    self.body = data[i + 4:end]
                    self._finish()
                    if end < len(data) and self.pending and not self.closed:
                        self.data_received(data[end:])  # pipelined responses behind it
                    return
                data = data[i + 4:]  # head consumed (or a bodiless response finished): general path
        self.buf += data
        while True:
            if not self.head_done:
                i = self.buf.find(_CRLF2)
                if i < 0:
                    return
                head = bytes(self.buf[:i])
                del self.buf[:i + 4]
                self._parse_head(head)
                if not self.head_done:  # a bodiless response completed inside _parse_head
                    if self.buf and self.pending:
                        continue
                    return
            if self.chunked:
                if not self._parse_chunks():
                    return
            elif self.clen >= 0:
                if self.stream is not None:
                    self._feed_stream(bytes(self.buf))
                    self.clen -= len(self.buf)
                    self.buf.clear()
                    if self.clen <= 0:
                        self._finish()
                    return
                if len(self.buf) < self.clen:
                    return
                self.body += self.buf[:self.clen]
                del self.buf[:self.clen]
                self._finish()
            else:  # read until close
                if self.stream is not None:
                    self._feed_stream(bytes(self.buf))
                else:
                    self.body += self.buf
                self.buf.clear()
                return
            if not self.buf or not self.pending or self.closed:
                return

    def _parse_head(self, head: bytes):
        if _parse_native is not None:
            try:
                status, clen, chunked, close, retry = _parse_native(head)
            except ValueError as e:
                raise E.TransportError(f"malformed response head: {e}") from e
            self.headers = _NO_HEADERS if retry is None else {"retry-after": retry}
        else:
            status, clen, chunked, close, self.headers = _parse_head_py(head)
        self.status = status
        self.head_done = True
        if chunked:
            self.chunked = True
        elif clen >= 0:
            self.clen = clen
        elif status in (204, 304) or 100 <= status < 200:
            self.clen = 0
        else:
            self.until_close = True
        if close:
            self.keep_alive = False
        if self.stream is not None and self.fut is not None and not self.fut.done():
            # streaming: hand the status/headers over now, body follows as lines
            self.fut.set_result(_Response(self.status, self.headers, b""))
        if self.clen == 0 and not self.chunked:
            self._finish()

    def _parse_chunks(self) -> bool:
        """Consume complete chunks; True once the terminating chunk (and trailers) were read."""
        buf = self.buf
        if self.stream is not None and _chunk_lines is not None:
            # a watch body: every complete line of what arrived, cut in one native pass (data taken before
            # its chunk is complete; chunk_left may then also be -3, the CRLF after a chunk's data)
            lines, self.chunk_left, used, done, self.linebuf = _chunk_lines(buf, self.chunk_left, self.linebuf)
            del buf[:used]
            if lines:
                self._emit(lines)
            if done:
                self._finish()
            return done
        while True:
            if self.chunk_left == -1:  # expecting a chunk-size line
                i = buf.find(b"\r\n")
                if i < 0:
                    return False
                size = int(bytes(buf[:i]).split(b";", 1)[0].strip(), 16)
                del buf[:i + 2]
                self.chunk_left = size if size else -2
            if self.chunk_left == -2:  # after the last chunk: trailer lines until an empty one
                j = buf.find(b"\r\n")
                if j < 0:
                    return False
                del buf[:j + 2]
                if j == 0:
                    self._finish()
                    return True
                continue
            if len(buf) < self.chunk_left + 2:
                return False
            data = bytes(buf[:self.chunk_left])
            del buf[:self.chunk_left + 2]
            self.chunk_left = -1
            if self.stream is not None:
                self._feed_stream(data)
            else:
                self.body += data

    def _feed_stream(self, data: bytes):
        lb = self.linebuf
        lb += data
        if b"\n" not in data:
            return
        parts = lb.split(b"\n")
        tail = parts.pop()
        self.linebuf = bytearray(tail)
        lines = [bytes(p) for p in parts if p]
        if lines:
            self._emit(lines)

    def _emit(self, lines: list) -> None:
        if self.line_tap is not None:
            self._tap(lines)
        self.stream.extend(lines)
        self.stream_event.set()
        if len(self.stream) > (self.HIGH_WATER if self.line_tap is None else self.TAPPED_HIGH_WATER) and \
                not self.paused and self.transport is not None:
            self.paused = True
            self.transport.pause_reading()

    def _tap(self, lines: list) -> None:
        try:
            self.line_tap(lines)
        except Exception:  # noqa: BLE001 — a tap must not break the stream its consumer reads
            import logging
            logging.getLogger("ncc.transport").exception("watch line tap failed")

    def _finish(self):
        if self.stream is not None:
            if self.linebuf.strip():
                line = bytes(self.linebuf)
                if self.line_tap is not None:
                    self._tap([line])
                self.stream.append(line)
                self.linebuf = bytearray()
            self.stream_done = True
            self.stream_event.set()
            return
        fut = self.pending.popleft() if self.pending else None
        resp = _Response(self.status, self.headers, bytes(self.body))
        keep = self.keep_alive
        self._reset()
        if fut is not None and not fut.done():
            fut.set_result(resp)
        if not keep or self.closed:
            self.close()  # connection_lost fails whatever was pipelined behind this response
        elif not self.pending:
            self.pool._release(self)

    # ---------------------------------------------------------------- API
    def send(self, data: bytes, stream: bool = False) -> asyncio.Future:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self.pending.append(fut)
        if stream:
            self.stream = deque()
            self.stream_event = asyncio.Event()
            self.transport.write(data)
            return fut
        if self.pool.pipeline_depth > 1:
            # requests queued on this connection in the same loop iteration leave in one write
            self._out.append(data)
            if self._flush_handle is None:
                self._flush_handle = loop.call_soon(self._flush)
        else:
            self.transport.write(data)
        return fut

    def _flush(self):
        self._flush_handle = None
        out, self._out = self._out, []
        if out and not self.closed and self.transport is not None:
            self.transport.write(out[0] if len(out) == 1 else b"".join(out))

    def resume(self):
        hw = self.HIGH_WATER if self.line_tap is None else self.TAPPED_HIGH_WATER
        if self.paused and self.transport is not None and self.stream is not None and \
                len(self.stream) < hw // 2:
            self.paused = False
            self.transport.resume_reading()

    def close(self):
        if not self.closed:
            self.closed = True
            if self.transport is not None:
                self.transport.close()


class ConnectionPool:
    def __init__(self, server: str, *, ssl_context: _ssl.SSLContext | None = None, server_hostname: str | None = None,
                 max_size: int = 64, connect_timeout: float = 10.0, pipeline_depth: int = 1,
                 proxy: str | None = None):
        u = urlsplit(server)
        self.proxy = proxy  # an HTTP CONNECT proxy (ncc/kube/proxy.py) every connection tunnels through
        self.scheme = u.scheme
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.host_header = u.netloc.encode()
        self.ssl = ssl_context if u.scheme == "https" else None
        self.server_hostname = server_hostname
        self.max_size = max_size
        self.connect_timeout = connect_timeout
        self.pipeline_depth = max(1, pipeline_depth)
        self._idle: list[_Conn] = []
        self._busy: set = set()  # open connections with requests in flight (pipelining candidates)
        self._connecting = 0
        self._wake: asyncio.Future | None = None
        self._limit = max_size * self.pipeline_depth
        self._inflight = 0
        self._slot_waiters: deque = deque()
        self._sweep_handle = None
        self.opened = 0

    async def _connect(self) -> _Conn:
        loop = asyncio.get_running_loop()
        kw = {}
        if self.ssl is not None:
            kw["ssl"] = self.ssl
            kw["server_hostname"] = self.server_hostname or self.host
        try:
            if self.proxy:
                from .proxy import open_tunnel
                sock = await open_tunnel(self.proxy, self.host, self.port, self.connect_timeout)
                coro = loop.create_connection(lambda: _Conn(self), sock=sock, **kw)
            else:
                coro = loop.create_connection(lambda: _Conn(self), self.host, self.port, **kw)
            _, proto = await wait_timeout(coro, self.connect_timeout)
        except (OSError, asyncio.TimeoutError, _ssl.SSLError) as e:
            raise E.TransportError(f"connect {self.host}:{self.port}: {type(e).__name__}: {e}") from e
        self.opened += 1
        return proto

    def _release(self, c: _Conn) -> None:
        self._busy.discard(c)
        if not c.closed:
            self._idle.append(c)

    def _discard(self, c: _Conn) -> None:
        self._busy.discard(c)
        try:
            self._idle.remove(c)
        except ValueError:
            pass

    async def _acquire(self) -> _Conn:
        while True:
            while self._idle:
                c = self._idle.pop()
                if not c.closed:
                    return c
            if self.pipeline_depth == 1 or len(self._busy) + self._connecting < self.max_size:
                break
            best = None
            for c in self._busy:
                if not c.closed and len(c.pending) < self.pipeline_depth and \
                        (best is None or len(c.pending) < len(best.pending)):
                    best = c
            if best is not None:
                return best
            if not self._connecting:
                break  # every connection died: open a fresh one
            if self._wake is None or self._wake.done():
                self._wake = asyncio.get_running_loop().create_future()
            await asyncio.shield(self._wake)  # a connect in progress completes (or fails): pick again
        self._connecting += 1
        try:
            c = await self._connect()
            self._busy.add(c)
            return c
        finally:
            self._connecting -= 1
            if self._wake is not None and not self._wake.done():
                self._wake.set_result(None)

    def _head(self, method: str, target: str, headers: dict, body_len: int | None, block: bytes | None = None) -> bytes:
        """Request line + headers.  `block` is the caller's pre-rendered "K: V\r\n" header section (the
        REST client memoises it per credential), so a steady-state request only formats its target."""
        if block is None:
            block = b"".join(f"{k}: {v}\r\n".encode("latin-1") for k, v in headers.items())
        host = b"" if "Host" in headers else b"Host: " + self.host_header + b"\r\n"
        clen = b"" if body_len is None else b"Content-Length: %d\r\n" % body_len
        return b"%s %s HTTP/1.1\r\n%s%s%s\r\n" % (method.encode(), target.encode(), host, block, clen)

    @staticmethod
    def _expire(c: _Conn, what: str) -> None:
        """Fail the in-flight exchange and drop the connection (request timeout).

        Timeouts are plain loop timers rather than `asyncio.wait_for`, which costs a Task per request
        and on Python 3.10 can swallow a concurrent cancellation (bpo-42130) — a hang at shutdown."""
        fut = c.fut
        c.timed_out = True
        if fut is not None and not fut.done():
            c.pending.popleft()
            fut.set_exception(E.TransportError(f"{what}: timed out"))
        c.close()

    # ---- request slots: at most max_size × pipeline_depth exchanges in flight (a counting semaphore
    # without asyncio.Semaphore's coroutine + waiter bookkeeping on the uncontended path)
    async def _take_slot(self) -> None:
        if self._inflight < self._limit and not self._slot_waiters:
            self._inflight += 1
            return
        fut = asyncio.get_running_loop().create_future()
        self._slot_waiters.append(fut)
        try:
            await fut  # the releasing request hands its slot over (no decrement/increment race)
        except BaseException:
            if fut.done() and not fut.cancelled():
                self._give_slot()  # woken, then cancelled before running: pass the slot on
            else:
                try:
                    self._slot_waiters.remove(fut)
                except ValueError:
                    pass
            raise

    def _give_slot(self) -> None:
        while self._slot_waiters:
            w = self._slot_waiters.popleft()
            if not w.done():
                w.set_result(None)
                return
        self._inflight -= 1

    # ---- timeouts: one coarse sweep per second over the busy connections instead of a timer per request
    def _arm_sweep(self) -> None:
        if self._sweep_handle is None:
            self._sweep_handle = asyncio.get_running_loop().call_later(self.SWEEP_PERIOD, self._sweep)

    def _sweep(self) -> None:
        self._sweep_handle = None
        now = asyncio.get_running_loop().time()
        for c in [c for c in self._busy if c.deadline is not None and c.deadline <= now]:
            if c.fut is not None and not c.fut.done():
                self._expire(c, c.deadline_what)
        if self._busy:
            self._arm_sweep()

    SWEEP_PERIOD = 0.5

    async def request(self, method: str, target: str, headers: dict, body: bytes | None,
                      timeout: float | None = 30.0, block: bytes | None = None) -> _Response:
        loop = asyncio.get_running_loop()
        await self._take_slot()
        try:
            for attempt in (0, 1):
                c = await self._acquire()
                reused = c.uses > 0
                c.uses += 1
                self._busy.add(c)
                data = self._head(method, target, headers, len(body) if body is not None else
                                  (0 if method in ("POST", "PUT", "PATCH") else None), block)
                if body:
                    data += body
                fut = c.send(data)
                timer = None
                if timeout:
                    if self.pipeline_depth == 1:  # one exchange per connection: the connection carries the deadline
                        c.deadline, c.deadline_what = loop.time() + timeout, f"{method} {target}"
                        self._arm_sweep()
                    else:
                        timer = loop.call_later(timeout, self._expire, c, f"{method} {target}")
                try:
                    return await fut
                except E.TransportError:
                    c.close()
                    # a reused keep-alive connection may have been closed by the server: retry once on a fresh
                    # one (never after a timeout: the server may have acted on the request)
                    if attempt == 0 and reused and not c.timed_out and not fut.cancelled():
                        continue
                    raise
                except BaseException:
                    c.close()
                    raise
                finally:
                    c.deadline = None
                    if timer is not None:
                        timer.cancel()
        finally:
            self._give_slot()
        raise E.TransportError("unreachable")  # pragma: no cover

    async def stream(self, target: str, headers: dict, timeout: float | None = None, batch: bool = False,
                     on_lines=None):
        """GET with a streaming body; yields complete lines (bytes) — or, with `batch`, lists of all the
        lines that arrived together, so the consumer iterates a plain list instead of resuming this
        generator per line.  Uses a dedicated connection.

        `timeout` bounds the whole stream (closing the connection ends it), like a client-side
        `timeoutSeconds`; waiting itself is a plain Event wait, so cancellation is never swallowed.
        `on_lines(lines)` (a successful stream only) sees every line as soon as it is read off the socket,
        before the consumer of this generator gets it."""
        c = await self._connect()
        loop = asyncio.get_running_loop()
        head_timer = loop.call_later(self.connect_timeout + 20, self._expire, c, f"GET {target}")
        stream_timer = None
        try:
            resp = await c.send(self._head("GET", target, headers, None), stream=True)
            head_timer.cancel()
            if timeout:
                stream_timer = loop.call_later(timeout, c.close)
            if resp.status >= 300:
                # drain the (small) error body
                while not c.stream_done:
                    c.stream_event.clear()
                    await c.stream_event.wait()
                raw = b"\n".join(c.stream) + bytes(c.linebuf)
                yield resp, raw
                return
            if on_lines is not None:
                if c.stream:
                    on_lines(list(c.stream))  # lines that came in with the response head
                c.line_tap = on_lines
            yield resp, None
            while True:
                if batch:
                    while c.stream:  # lines may arrive while the consumer works on a batch: drain them all
                        lines = list(c.stream)
                        c.stream.clear()
                        c.resume()
                        yield None, lines
                else:
                    while c.stream:
                        yield None, c.stream.popleft()
                        c.resume()
                if c.stream_done or c.closed:
                    return
                c.stream_event.clear()
                await c.stream_event.wait()
        finally:
            head_timer.cancel()
            if stream_timer is not None:
                stream_timer.cancel()
            c.close()

    def close(self) -> None:
        if self._sweep_handle is not None:
            self._sweep_handle.cancel()
            self._sweep_handle = None
        for c in list(self._idle) + list(self._busy):
            c.close()
        self._idle.clear()
        self._busy.clear()
