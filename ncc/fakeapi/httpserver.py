"""Minimal HTTP/1.1 server on asyncio Protocols for the fake kube-apiserver.

A real kube-apiserver is a multi-core Go process that sustains tens of thousands of writes per
second; a benchmark substrate that spends ~150 µs of Python per request in a generic web
framework would make the *substrate* the bottleneck of every fan-out measurement.  This server
implements exactly what the fake apiserver needs — keep-alive connections, Content-Length
request bodies, Content-Length responses and chunked streaming responses (watches) with write
back-pressure — with one Python-level pass over each request head.

The handler API mirrors the subset of aiohttp.web the fake apiserver was written against
(`request.path/.method/.query/.headers/.content_type/.read()`, `Response`, `StreamResponse`).
"""
from __future__ import annotations

import asyncio
import json
from urllib.parse import parse_qsl, unquote

from . import native as _native

_CRLF2 = b"\r\n\r\n"
_HEADS: dict = {}
_REASONS = {200: "OK", 201: "Created", 204: "No Content", 400: "Bad Request", 401: "Unauthorized",
            403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed", 409: "Conflict", 410: "Gone",
            415: "Unsupported Media Type", 422: "Unprocessable Entity", 429: "Too Many Requests",
            500: "Internal Server Error", 503: "Service Unavailable", 504: "Gateway Timeout"}


_QUERY_MEMO: dict = {}  # raw query → parsed (write requests repeat e.g. "fieldManager=…"); read-only use


class Request:
    __slots__ = ("method", "path", "raw_query", "headers", "body", "_query", "_conn", "_h2")

    def __init__(self, method: str, target: str, headers: dict, body: bytes):
        self.method = method
        path, _, q = target.partition("?")
        self.path = unquote(path)
        self.raw_query = q
        self.headers = headers
        self.body = body
        self._query = None
        self._h2 = None  # (H2Connection, stream) when it came over HTTP/2 (ncc/fakeapi/h2.py)

    @property
    def query(self) -> dict:
        if self._query is None:
            q = _QUERY_MEMO.get(self.raw_query)
            if q is None:
                q = dict(parse_qsl(self.raw_query, keep_blank_values=True))
                if len(_QUERY_MEMO) < 1024 and "resourceVersion" not in q and "continue" not in q:
                    _QUERY_MEMO[self.raw_query] = q
            self._query = q
        return self._query

    @property
    def content_type(self) -> str:
        return self.headers.get("content-type", "application/octet-stream").split(";", 1)[0].strip()

    @property
    def can_read_body(self) -> bool:
        return bool(self.body)

    async def read(self) -> bytes:
        return self.body


class Response:
    __slots__ = ("status", "body", "content_type", "headers")

    def __init__(self, status: int = 200, body: bytes | None = None, text: str | None = None,
                 content_type: str | None = None, headers: dict | None = None):
        self.status = status
        if text is not None:
            body = text.encode()
            content_type = content_type or "text/plain"
        self.body = body or b""
        self.content_type = content_type or "application/json"
        self.headers = headers or {}

    def encode(self) -> bytes:
        if not self.headers:
            head = _HEADS.get((self.status, self.content_type))
            if head is None:
                head = _HEADS[(self.status, self.content_type)] = (
                    f"HTTP/1.1 {self.status} {_REASONS.get(self.status, 'Status')}\r\n"
                    f"Content-Type: {self.content_type}\r\nContent-Length: ").encode()
            return b"%s%d\r\n\r\n%s" % (head, len(self.body), self.body)
        h = [f"HTTP/1.1 {self.status} {_REASONS.get(self.status, 'Status')}", f"Content-Type: {self.content_type}",
             f"Content-Length: {len(self.body)}"]
        for k, v in self.headers.items():
            h.append(f"{k}: {v}")
        return ("\r\n".join(h) + "\r\n\r\n").encode() + self.body


class Deferred:
    """A response `fast` handlers answer later, from a callback (no task): the connection waits for it."""
    __slots__ = ("response", "_cb")

    def __init__(self):
        self.response = None
        self._cb = None

    def resolve(self, response: Response) -> None:
        self.response = response
        cb, self._cb = self._cb, None
        if cb is not None:
            cb(response)

    def then(self, cb) -> None:
        self._cb = cb


def json_response(obj, status: int = 200) -> Response:
    return Response(status=status, body=json.dumps(obj, separators=(",", ":")).encode())


class StreamResponse:
    """Chunked streaming response (watch).  `prepare` sends the head; `write` sends one chunk."""

    def __init__(self, status: int = 200, headers: dict | None = None):
        self.status = status
        self.headers = {k: v for k, v in (headers or {}).items() if k.lower() != "transfer-encoding"}
        self._conn: "_ServerConn | None" = None
        self._h2w = None
        self.prepared = False

    async def prepare(self, request: Request) -> None:
        conn = request._conn  # type: ignore[attr-defined]
        self._conn = conn
        if request._h2 is not None:  # HTTP/2: HEADERS now, DATA frames per write, END_STREAM at EOF
            from .h2 import H2StreamWriter
            self._h2w = H2StreamWriter(*request._h2)
            self._h2w.prepare(self.status, self.headers)
            self.prepared = True
            return
        h = [f"HTTP/1.1 {self.status} {_REASONS.get(self.status, 'Status')}", "Transfer-Encoding: chunked"]
        for k, v in self.headers.items():
            h.append(f"{k}: {v}")
        conn.transport.write(("\r\n".join(h) + "\r\n\r\n").encode())
        self.prepared = True

    async def write(self, data: bytes) -> None:
        c = self._conn
        if c is None or c.closed:
            raise ConnectionResetError("client went away")
        if self._h2w is not None:
            if data:
                self._h2w.write(data)
        elif data:
            c.transport.write(b"%x\r\n%s\r\n" % (len(data), data))
        await c.drain()

    async def write_eof(self) -> None:
        c = self._conn
        if c is not None and not c.closed:
            if self._h2w is not None:
                self._h2w.write_eof()
            else:
                c.transport.write(b"0\r\n\r\n")


class _ServerConn(asyncio.Protocol):
    def __init__(self, server: "HttpServer"):
        self.server = server
        self.transport = None
        self.buf = bytearray()
        self.closed = False
        self.busy = False
        self.api = False  # served a request other than a watch (connection statistics)
        self._drain: asyncio.Future | None = None
        self.h2 = None  # ncc/fakeapi/h2.py H2Connection once the connection speaks HTTP/2
        self.fresh = True  # nothing received yet (an HTTP/2 preface can only come first)

    def connection_made(self, transport):
        self.transport = transport
        srv = self.server
        srv._conns.add(self)
        srv.accepted += 1
        ssl_obj = transport.get_extra_info("ssl_object")
        if srv.http2 and ssl_obj is not None and ssl_obj.selected_alpn_protocol() == "h2":
            self._start_h2()

    def _start_h2(self):
        from .h2 import H2Connection
        self.h2 = H2Connection(self, self.server)
        self.api = True
        srv = self.server
        srv.api_conns += 1
        srv.max_api_conns = max(srv.max_api_conns, srv.api_conns)

    def connection_lost(self, exc):
        self.closed = True
        srv = self.server
        srv._conns.discard(self)
        if self.api:
            srv.api_conns -= 1
        if self.h2 is not None:
            self.h2.connection_lost()
        if self._drain is not None and not self._drain.done():
            self._drain.set_result(None)

    def pause_writing(self):
        if self._drain is None or self._drain.done():
            self._drain = asyncio.get_running_loop().create_future()

    def resume_writing(self):
        if self._drain is not None and not self._drain.done():
            self._drain.set_result(None)

    async def drain(self):
        if self._drain is not None and not self._drain.done():
            await self._drain

    def data_received(self, data: bytes):
        if self.h2 is not None:
            self.h2.data_received(data)
            return
        if self.fresh:
            self.fresh = False
            if self.server.http2 and data[:4] == b"PRI ":  # HTTP/2 with prior knowledge (cleartext)
                self._start_h2()
                self.h2.data_received(data)
                return
        self.buf += data
        if not self.busy:
            self._next()

    def _next(self):
        fast = self.server.fast
        while True:
            buf = self.buf
            i = buf.find(_CRLF2)
            if i < 0:
                if len(buf) > 1 << 20:
                    self.transport.close()
                return
            try:
                method, target, headers = _parse_head(bytes(buf[:i]))
                clen = int(headers.get("content-length", "0") or 0)
            except ValueError:
                self.transport.close()
                return
            if len(buf) < i + 4 + clen:
                return  # wait for the full body
            body = bytes(buf[i + 4:i + 4 + clen])
            del buf[:i + 4 + clen]
            req = Request(method, target, headers, body)
            req._conn = self  # type: ignore[attr-defined]
            if not self.api and "watch=" not in target:
                self.api = True
                srv = self.server
                srv.api_conns += 1
                if srv.api_conns > srv.max_api_conns:
                    srv.max_api_conns = srv.api_conns
            keep = headers.get("connection", "").lower() != "close"
            if fast is not None:
                try:
                    resp = fast(req)
                except Exception as e:  # noqa: BLE001
                    resp = Response(500, text=f"internal error: {e}")
                if isinstance(resp, Deferred):
                    if resp.response is None:  # answered later from a callback: wait for it, in order
                        self.busy = True
                        resp.then(lambda r, k=keep: self._deferred_done(r, k))
                        return
                    resp = resp.response
                if resp is not None:  # answered synchronously: no task, keep parsing pipelined requests
                    self.transport.write(resp.encode())
                    if not keep:
                        self.transport.close()
                        return
                    continue
            self.busy = True
            task = asyncio.ensure_future(self.server.handler(req))
            task.add_done_callback(lambda t, k=keep: self._done(t, k))
            return

    def _deferred_done(self, resp: Response, keep: bool) -> None:
        self.busy = False
        if self.closed:
            return
        self.transport.write(resp.encode())
        if not keep:
            self.transport.close()
            return
        if self.buf:
            self._next()

    def _done(self, task: asyncio.Task, keep: bool):
        self.busy = False
        if self.closed:
            return
        try:
            resp = task.result()
        except Exception as e:  # noqa: BLE001
            resp = Response(500, text=f"internal error: {e}")
        if isinstance(resp, Response):
            self.transport.write(resp.encode())
        if not keep:
            self.transport.close()
            return
        if self.buf:
            self._next()


def _parse_head_py(head: bytes) -> tuple:
    lines = head.split(b"\r\n")
    method, target, _ = lines[0].decode("latin-1").split(" ", 2)
    headers = {}
    for ln in lines[1:]:
        k, sep, v = ln.partition(b":")
        if sep:  # a line without a colon is not a header
            headers[k.strip().lower().decode("latin-1")] = v.strip().decode("latin-1")
    return method, target, headers


_native_mod = _native.load()
_parse_head = getattr(_native_mod, "parse_request_head", None) or _parse_head_py


class HttpServer:
    def __init__(self, handler, fast=None):
        """`handler(request)` is a coroutine; optional `fast(request)` answers synchronously or returns None."""
        self.handler = handler
        self.fast = fast
        self._server: asyncio.AbstractServer | None = None
        self._conns: set = set()
        self.port: int | None = None
        self.accepted = 0  # connections accepted so far
        self.api_conns = self.max_api_conns = 0  # open connections that served a non-watch request; the most at once
        self.http2 = False  # accept HTTP/2: ALPN "h2" on TLS (the context must offer it), prior knowledge on TCP
        self.h2_options: dict = {}  # h2_max_streams, h2_goaway_after (ncc/fakeapi/h2.py)
        self.h2_stats = {"connections": 0, "streams": 0, "max_open": 0, "refused": 0, "goaways": 0, "malformed": 0}

    def conn_stats(self) -> dict:
        return {"open": len(self._conns), "accepted": self.accepted, "api_open": self.api_conns,
                "api_max": self.max_api_conns, "h2": dict(self.h2_stats)}

    async def start(self, host: str, port: int, ssl_context=None) -> int:
        loop = asyncio.get_running_loop()
        self._server = await loop.create_server(lambda: _ServerConn(self), host, port, ssl=ssl_context, backlog=1024)
        self.port = self._server.sockets[0].getsockname()[1]
        return self.port

    async def stop(self) -> None:
        if self._server is not None:
            self._server.close()
            for c in list(self._conns):
                if c.transport is not None:
                    c.transport.close()
            await self._server.wait_closed()
            self._server = None
