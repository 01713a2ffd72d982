"""REST client for kube-apiservers: one keep-alive connection pool per cluster.

Two interchangeable transports: `fast` (default; raw asyncio protocols, `ncc.kube.transport`)
and `aiohttp`.

This is the "distributed communication backend" of the system: JSON over
HTTP(S) to kube-apiservers, with TLS and credentials from kubeconfig (CA, client cert/key,
bearer token, token file, exec plugin), a bounded keep-alive pool sized for fan-out
concurrency, chunked JSON-lines watch streams, typed errors, `Retry-After`-driven retries of
throttled/unavailable responses (client-go `rest.Request` semantics) and one credential
refresh on 401 for exec-plugin users.
"""
from __future__ import annotations

import asyncio
import json
import os
import ssl
import tempfile
from typing import AsyncIterator
from urllib.parse import urlencode


class _LazyModule:
    """Import on first attribute access: aiohttp costs ~0.2 s of process start-up and only the optional
    `transport: aiohttp` path uses it (every executor process starts with this module)."""

    def __init__(self, name: str):
        self._name = name

    def __getattr__(self, attr):
        import importlib
        mod = importlib.import_module(self._name)
        globals()[self._name] = mod
        return getattr(mod, attr)


aiohttp = _LazyModule("aiohttp")

from .. import native as _native
from ..api.jsonenc import dumps_bytes, loads_fast
from ..api.resources import ResourceType
from . import errors as E
from . import h2client
from .client import PATCH_MERGE, KubeClient, WatchEvent
from .kubeconfig import ClusterConfig, CredentialSource
from .proxy import proxy_for
from .transport import ConnectionPool

USER_AGENT = "nexus-configuration-controller/ncc (linux/amd64)"
_JSON = "application/json"


def _ssl_context(cfg: ClusterConfig, exec_cert: tuple | None = None) -> ssl.SSLContext | bool:
    if not cfg.is_tls:
        return False
    ctx = ssl.create_default_context()
    if cfg.insecure:
        ctx.check_hostname = False
        ctx.verify_mode = ssl.CERT_NONE
    elif cfg.ca_data:
        ctx.load_verify_locations(cadata=cfg.ca_data.decode())
    cert = exec_cert or ((cfg.client_cert_data, cfg.client_key_data)
                         if cfg.client_cert_data and cfg.client_key_data else None)
    if cert:
        # ssl needs files for the key pair; keep them private and short-lived.
        with tempfile.TemporaryDirectory(prefix="ncc-tls-") as d:
            cp, kp = os.path.join(d, "tls.crt"), os.path.join(d, "tls.key")
            for p, data in ((cp, cert[0]), (kp, cert[1])):
                fd = os.open(p, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
                with os.fdopen(fd, "wb") as f:
                    f.write(data)
            ctx.load_cert_chain(cp, kp)
    return ctx


_QUERY_CACHE: dict = {}


def _query(params: dict) -> str:
    """"?k=v&…" for the non-None params; memoised (writes repeat the same fieldManager/dryRun sets)."""
    key = tuple(params.items())
    try:
        return _QUERY_CACHE[key]
    except KeyError:
        pass
    except TypeError:  # unhashable value
        key = None
    q = {k: v for k, v in params.items() if v is not None}
    out = ("?" + urlencode(q)) if q else ""
    if key is not None and len(_QUERY_CACHE) < 4096:
        _QUERY_CACHE[key] = out
    return out


_scan_object = getattr(_native.load(), "scan_object", None)
_members_equal = getattr(_native.load(), "members_equal", None)


class RestClient(KubeClient):
    def __init__(self, cfg: ClusterConfig, *, pool_size: int = 64, request_timeout: float = 30.0,
                 max_retries: int = 5, cluster_name: str | None = None, transport: str = "fast",
                 pipeline_depth: int = 1, http2: str = "auto"):
        if transport not in ("fast", "aiohttp"):
            raise ValueError(f"unknown transport {transport!r}")
        if http2 not in ("off", "auto", "on"):
            raise ValueError(f"unknown http2 mode {http2!r}")
        self.transport = transport
        self.http2 = http2
        self._pool: ConnectionPool | None = None
        self.cfg = cfg
        self.cluster_name = cluster_name or cfg.name or cfg.server
        self.pool_size = pool_size
        self.pipeline_depth = pipeline_depth
        self.request_timeout = request_timeout
        self.max_retries = max_retries
        self.creds = CredentialSource(cfg)
        self._hdr_cache: dict = {}
        self._session: aiohttp.ClientSession | None = None
        self._session_lock = asyncio.Lock()
        self.stats = {"requests": 0, "retries": 0, "errors": 0, "watch_streams": 0}
        # kubeconfig proxy-url, else client-go's HTTPS_PROXY / HTTP_PROXY / NO_PROXY (ncc/kube/proxy.py)
        self.proxy = proxy_for(cfg.server, cfg.proxy_url)
        if self.proxy and self.proxy.startswith("socks") and transport != "fast":
            raise ValueError("a socks5 proxy needs the fast transport (aiohttp speaks only http:// proxies)")

    async def _get_session(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            async with self._session_lock:
                if self._session is None or self._session.closed:
                    exec_cert = await self.creds.exec_client_cert()
                    ctx = _ssl_context(self.cfg, exec_cert)
                    conn = aiohttp.TCPConnector(limit=self.pool_size, limit_per_host=self.pool_size, ssl=ctx,
                                                ttl_dns_cache=300, keepalive_timeout=60,
                                                enable_cleanup_closed=False)
                    self._session = aiohttp.ClientSession(connector=conn, json_serialize=json.dumps,
                                                          headers={"User-Agent": USER_AGENT, "Accept": _JSON},
                                                          skip_auto_headers=("Accept-Encoding",))
        return self._session

    async def _get_pool(self) -> ConnectionPool:
        if self._pool is None:
            async with self._session_lock:
                if self._pool is None:
                    exec_cert = await self.creds.exec_client_cert()
                    ctx = _ssl_context(self.cfg, exec_cert)
                    kw = dict(ssl_context=ctx or None, server_hostname=self.cfg.tls_server_name,
                              max_size=self.pool_size, connect_timeout=self.request_timeout,
                              pipeline_depth=self.pipeline_depth, proxy=self.proxy)
                    tls = self.cfg.server.startswith("https:")
                    if h2client.AVAILABLE and (self.http2 == "on" or (self.http2 == "auto" and tls)):
                        # client-go's transport: HTTP/2 negotiated by ALPN (prior knowledge on cleartext with "on")
                        self._pool = h2client.H2Pool(self.cfg.server, prior_knowledge=self.http2 == "on",
                                                     fallback_ssl_context=_ssl_context(self.cfg, exec_cert) or None,
                                                     **kw)
                    else:
                        self._pool = ConnectionPool(self.cfg.server, **kw)
        return self._pool

    @property
    def protocol(self) -> str | None:
        """"h2" or "http/1.1" once the first connection is made (None before, or with the aiohttp transport)."""
        pool = self._pool
        if pool is None:
            return None
        return pool.protocol if isinstance(pool, h2client.H2Pool) else "http/1.1"

    async def _send(self, method: str, target: str, headers: dict, data, block: bytes | None = None):
        """One HTTP exchange → (status, raw body, Retry-After header or None).  `block` is the pre-rendered
        header section of `headers` (fast transport)."""
        if self.transport == "fast":
            pool = self._pool or await self._get_pool()
            body = data.encode() if isinstance(data, str) else data
            resp = await pool.request(method, target, headers, body, timeout=self.request_timeout, block=block)
            return resp.status, resp.body, resp.headers.get("retry-after")
        session = await self._get_session()
        try:
            async with session.request(method, self.cfg.server + target, data=data, headers=headers, proxy=self.proxy,
                                       timeout=aiohttp.ClientTimeout(total=self.request_timeout)) as resp:
                raw = await resp.read()
                return resp.status, raw, resp.headers.get("Retry-After")
        except (aiohttp.ClientConnectionError, aiohttp.ClientPayloadError, asyncio.TimeoutError, OSError) as e:
            raise E.TransportError(f"{method} {target}: {type(e).__name__}: {e}") from e

    async def _headers(self, content_type: str | None, refresh: bool = False) -> dict:
        return self._render_headers(content_type, await self.creds.token(force_refresh=refresh))[0]

    def _headers_now(self, content_type: str | None) -> tuple | None:
        """(headers, rendered header block) without awaiting when the credential is at hand; memoised per
        (content type, token), so steady-state requests build no header dict and no header bytes."""
        hit, tok = self.creds.cached_token()
        if not hit:
            return None
        key = (content_type, tok)
        got = self._hdr_cache.get(key)
        if got is None:
            if len(self._hdr_cache) > 16:  # rotated tokens: keep the cache small
                self._hdr_cache.clear()
            got = self._hdr_cache[key] = self._render_headers(content_type, tok)
        return got

    def _render_headers(self, content_type: str | None, tok: str | None) -> tuple:
        h = {"User-Agent": USER_AGENT, "Accept": _JSON}
        if content_type:
            h["Content-Type"] = content_type
        if tok:
            h["Authorization"] = f"Bearer {tok}"
        elif self.cfg.username is not None:
            import base64
            h["Authorization"] = "Basic " + base64.b64encode(
                f"{self.cfg.username}:{self.cfg.password or ''}".encode()).decode()
        if self.cfg.tls_server_name:
            h["Host"] = self.cfg.tls_server_name
        block = b"".join(f"{k}: {v}\r\n".encode("latin-1") for k, v in h.items())
        return h, block

    async def request(self, method: str, path: str, *, params: dict | None = None, body=None,
                      content_type: str = _JSON, raw: bool = False):
        """One API call with auth refresh and Retry-After retries → decoded JSON (or the raw body bytes
        of a successful response with `raw=True`); non-2xx raises the matching ApiError."""
        target = path
        if params:
            target += _query(params)
        data = None
        if body is not None:
            data = body if isinstance(body, (bytes, str)) else dumps_bytes(body)
        return await self._exchange(method, target, data, content_type if data is not None else None, raw)

    async def _exchange(self, method: str, target: str, data, ctype: str | None, raw_out: bool,
                        first: tuple | None = None):
        """The request loop behind `request`: send, then retry on 401 (credential refresh) and on
        throttling/unavailability with Retry-After.  `first` is a response already received for this
        request by a caller's fast path, handled before anything is re-sent."""
        refreshed = False
        attempt = 0
        while True:
            if first is not None:
                (status, body_bytes, retry_after), first = first, None
            else:
                self.stats["requests"] += 1
                got = None if refreshed else self._headers_now(ctype)
                if got is None:
                    got = self._render_headers(ctype, await self.creds.token())
                try:
                    status, body_bytes, retry_after = await self._send(method, target, got[0], data, got[1])
                except E.TransportError:
                    self.stats["errors"] += 1
                    raise
            if status < 300:
                if raw_out:
                    return bytes(body_bytes)
                return loads_fast(body_bytes) if body_bytes else None
            if status == 401 and (self.cfg.exec is not None or self.cfg.token_file) and not refreshed:
                refreshed = True
                await self.creds.token(force_refresh=True)
                continue
            if status in (429, 500, 502, 503, 504) and retry_after is not None and attempt < self.max_retries:
                attempt += 1
                self.stats["retries"] += 1
                try:
                    delay = min(float(retry_after), 10.0)
                except ValueError:
                    delay = 1.0
                await asyncio.sleep(delay)
                continue
            self.stats["errors"] += 1
            try:
                st = json.loads(body_bytes) if body_bytes else None
            except ValueError:
                st = None
            err = E.from_status(status, st if isinstance(st, dict) else None,
                                fallback_message=bytes(body_bytes[:200]).decode(errors="replace"))
            if retry_after is not None:
                try:
                    err.retry_after = float(retry_after)
                except ValueError:
                    pass
            raise err

    # ------------------------------------------------------------------ verbs
    async def get(self, rt, namespace, name):
        return await self.request("GET", rt.item_path(namespace, name))

    async def list(self, rt, namespace, *, label_selector=None, limit=None, continue_token=None,
                   resource_version=None):
        return await self.request("GET", rt.base_path(namespace), params={
            "labelSelector": label_selector, "limit": limit, "continue": continue_token,
            "resourceVersion": resource_version})

    async def create(self, rt, namespace, obj, *, field_manager=None):
        return await self.request("POST", rt.base_path(namespace), params={"fieldManager": field_manager}, body=obj)

    async def update(self, rt, namespace, obj, *, field_manager=None):
        name = (obj.get("metadata") or {}).get("name", "")
        return await self.request("PUT", rt.item_path(namespace, name), params={"fieldManager": field_manager},
                                  body=obj)

    async def update_status(self, rt, namespace, obj, *, field_manager=None):
        name = (obj.get("metadata") or {}).get("name", "")
        return await self.request("PUT", rt.item_path(namespace, name, "status"),
                                  params={"fieldManager": field_manager}, body=obj)

    async def patch(self, rt, namespace, name, body, *, patch_type=PATCH_MERGE, field_manager=None, force=None,
                    subresource=None):
        params = {"fieldManager": field_manager}
        if force is not None:
            params["force"] = "true" if force else "false"
        return await self.request("PATCH", rt.item_path(namespace, name, subresource), params=params, body=body,
                                  content_type=patch_type)

    async def write_meta(self, verb: str, rt, namespace, body: dict, *, name: str | None = None,
                         field_manager=None, patch_type=None, force=None, verify: tuple | None = None) -> tuple:
        """create/update/patch that returns only (namespace, name, resourceVersion, uid) of the stored object,
        read from the response by the native scanner instead of decoding it (slim-cache writers publish
        their own request body; the server's echo of the payload is not needed).

        `verify=(member, ...)` appends a fifth element: None when those top-level members of the response
        are byte-identical to the request's (the server stored what we sent), else the decoded response —
        the server rewrote the payload (CRD defaulting or pruning, a mutating webhook, or merely another
        encoding of the same JSON) and the caller must publish what was stored, not what it sent."""
        params = {"fieldManager": field_manager}
        if verb == "create":
            method, path = "POST", rt.base_path(namespace)
        elif verb == "update":
            method, path = "PUT", rt.item_path(namespace, name or (body.get("metadata") or {}).get("name", ""))
        else:
            method, path = "PATCH", rt.item_path(namespace, name)
            if force is not None:
                params["force"] = "true" if force else "false"
        ctype = patch_type if verb == "patch" else _JSON
        data = dumps_bytes(body)
        target = path + _query(params)
        pool = self._pool
        got = self._headers_now(ctype) if pool is not None and self.transport == "fast" else None
        if got is not None:
            # hot path (every shard write of an executor): straight onto the connection pool
            self.stats["requests"] += 1
            try:
                resp = await pool.request(method, target, got[0], data, timeout=self.request_timeout, block=got[1])
            except E.TransportError:
                self.stats["errors"] += 1
                raise
            raw = resp.body if resp.status < 300 else await self._exchange(
                method, target, data, ctype, True, first=(resp.status, resp.body, resp.headers.get("retry-after")))
        else:
            raw = await self._exchange(method, target, data, ctype, True)
        raw = bytes(raw) if not isinstance(raw, bytes) else raw
        stored = None
        if verify is not None and (_members_equal is None or not _members_equal(data, raw, verify)):
            stored = json.loads(raw)
        sc = _scan_object(raw) if _scan_object is not None else None
        if sc is None:
            m = ((stored if stored is not None else json.loads(raw)) or {}).get("metadata") or {}
            sc = (m.get("namespace", ""), m.get("name", ""), m.get("resourceVersion", ""), m.get("uid", ""))
        return sc if verify is None else sc + (stored,)

    async def delete(self, rt, namespace, name, *, propagation_policy=None, preconditions=None):
        body = None
        if propagation_policy or preconditions:
            body = {"kind": "DeleteOptions", "apiVersion": "v1"}
            if propagation_policy:
                body["propagationPolicy"] = propagation_policy
            if preconditions:
                body["preconditions"] = preconditions
        return await self.request("DELETE", rt.item_path(namespace, name), body=body)

    async def watch_raw(self, rt: ResourceType, namespace, *, resource_version=None, timeout_seconds=None,
                        allow_bookmarks=True, label_selector=None) -> AsyncIterator[bytes]:
        """The watch stream as raw JSON lines (one event per line), undecoded."""
        async for lines in self.watch_raw_batches(rt, namespace, resource_version=resource_version,
                                                  timeout_seconds=timeout_seconds, allow_bookmarks=allow_bookmarks,
                                                  label_selector=label_selector):
            for line in lines:
                yield line

    supports_line_tap = True  # watch_raw_batches(on_lines=...)

    async def watch_raw_batches(self, rt: ResourceType, namespace, *, resource_version=None, timeout_seconds=None,
                                allow_bookmarks=True, label_selector=None, on_lines=None) -> AsyncIterator[list]:
        """The watch stream as lists of raw JSON lines: everything that arrived in one read, undecoded.
        `on_lines(lines)` sees every line first — with the fast transport as soon as it is read off the
        socket, whatever the consumer of this generator is doing."""
        params = {"watch": "1", "resourceVersion": resource_version, "timeoutSeconds": timeout_seconds,
                  "allowWatchBookmarks": "true" if allow_bookmarks else None, "labelSelector": label_selector}
        target = rt.base_path(namespace) + "?" + urlencode({k: v for k, v in params.items() if v is not None})
        self.stats["watch_streams"] += 1
        headers = await self._headers(None)
        if self.transport == "fast":
            pool = await self._get_pool()
            stream = pool.stream(target, headers, timeout=(timeout_seconds + 30) if timeout_seconds else None,
                                 batch=True, on_lines=on_lines)
            try:
                async for resp, lines in stream:
                    if resp is not None:
                        if resp.status >= 300:
                            try:
                                st = json.loads(lines) if lines else None
                            except ValueError:
                                st = None
                            raise E.from_status(resp.status, st if isinstance(st, dict) else None)
                        continue
                    yield lines
            finally:
                await stream.aclose()
            return
        session = await self._get_session()
        url = self.cfg.server + target
        client_timeout = aiohttp.ClientTimeout(total=(timeout_seconds + 30) if timeout_seconds else None,
                                               sock_connect=self.request_timeout)
        try:
            async with session.get(url, headers=headers, timeout=client_timeout, proxy=self.proxy) as resp:
                if resp.status >= 300:
                    raw = await resp.read()
                    try:
                        st = json.loads(raw)
                    except ValueError:
                        st = None
                    raise E.from_status(resp.status, st if isinstance(st, dict) else None)
                buf = b""
                async for chunk in resp.content.iter_any():
                    buf += chunk
                    if b"\n" not in chunk:
                        continue
                    lines = buf.split(b"\n")
                    buf = lines.pop()
                    lines = [ln for ln in lines if ln]
                    if lines:
                        if on_lines is not None:
                            on_lines(lines)
                        yield lines
                if buf.strip():
                    if on_lines is not None:
                        on_lines([buf])
                    yield [buf]
        except (aiohttp.ClientConnectionError, aiohttp.ClientPayloadError, asyncio.TimeoutError, OSError) as e:
            raise E.TransportError(f"watch {url}: {type(e).__name__}: {e}") from e

    async def watch(self, rt: ResourceType, namespace, *, resource_version=None, timeout_seconds=None,
                    allow_bookmarks=True, label_selector=None) -> AsyncIterator[WatchEvent]:
        loads = loads_fast
        async for line in self.watch_raw(rt, namespace, resource_version=resource_version,
                                         timeout_seconds=timeout_seconds, allow_bookmarks=allow_bookmarks,
                                         label_selector=label_selector):
            ev = loads(line)
            yield WatchEvent(ev.get("type", ""), ev.get("object") or {})

    async def close(self) -> None:
        if self._pool is not None:
            self._pool.close()
            self._pool = None
        if self._session is not None and not self._session.closed:
            await self._session.close()
        self._session = None
