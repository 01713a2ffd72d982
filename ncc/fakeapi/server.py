"""HTTP front-end of the fake kube-apiserver (lean asyncio HTTP/1.1 server), over `ClusterState`.

Serves the REST surface the controller uses — core `/api/v1` and CRD `/apis/{group}/{version}`
paths, namespaced and cluster-wide, `GET` (get / list / `?watch=1`), `POST`, `PUT`
(incl. `/status`), `PATCH` (merge, strategic, json, apply) and `DELETE` — with Kubernetes
`Status` error bodies, chunked JSON-lines watch streams with periodic `BOOKMARK`s, and
`timeoutSeconds`.  It replaces envtest/kind for tests and benchmarks.

Test/bench control endpoints (not part of the Kubernetes API):
  GET  /_fake/stats    request counters and object counts
  POST /_fake/faults   {"latency_ms", "jitter_ms", "error_rate", "error_code", "throttle_rate",
                        "down", "drop_watches", "compact", "relist" (compact past every client's
                        revision, then drop every watch: each informer must relist), "rules", and the
                        request-admission model
                        "max_mutating_inflight", "apf_seats", "apf_queue", "apf_queue_wait_s",
                        "service_ms", "read_service_ms" (ncc/fakeapi/flowcontrol.py)} — fault injection for the
                       retry/backoff benchmark (BASELINE.json config 5) and for targeted tests:
                       `rules` = [{"method", "resource", "name", "code", "reason", "count",
                       "retry_after", "after"}, ...] fail the matching requests ("*" or absent = any;
                       `count` answers, -1 = until cleared; `retry_after` seconds go out as a Retry-After
                       header; `after`: serve the request, then answer with the error)
  GET  /_fake/writes   the mutating requests served so far ([method, plural, name, subresource, status,
                       monotonic time])
  POST /_fake/objects  bulk create `{"items": [...]}` without per-request overhead (bench seeding)
  POST /_fake/apply    `{"items": [...], "yield_every": n}` create-or-update a wave of user changes,
                       committed in slices of n with watch delivery in between; `{"staged": id}`
                       commits a body sent earlier to
  POST /_fake/stage    `{"id": id, "items": [...], ...}` (decoded ahead of a timed apply)
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import random
import signal
import ssl
import time

from . import httpserver as web

from ..api import resources as R
from ..api.jsonenc import dumps_bytes, loads_bytes
from ..aio import wait_timeout
from ..kube import errors as E
from ..kube.client import PATCH_APPLY, PATCH_JSON, PATCH_MERGE, PATCH_STRATEGIC
from .flowcontrol import FlowControl
from .markers import MarkerTracker
from .storage import ClusterState

log = logging.getLogger("ncc.fakeapi")

_JSON = "application/json"


def _dumps(o) -> bytes:
    return dumps_bytes(o)


def _status_response(err: E.ApiError) -> web.Response:
    headers = {}
    if err.retry_after is not None:
        headers["Retry-After"] = str(int(err.retry_after))
    return web.Response(status=err.code or 500, body=_dumps(err.status_object()), content_type=_JSON,
                        headers=headers)


class Faults:
    def __init__(self):
        self.latency_ms = 0.0
        self.jitter_ms = 0.0
        self.error_rate = 0.0
        self.error_code = 500
        self.throttle_rate = 0.0
        self.down = False
        self.write_only = True  # error_rate applies to mutating requests only
        self.rules: list[dict] = []  # targeted failures (see the module docstring)
        # request admission (flowcontrol.py): 0 = off
        self.max_mutating_inflight = 0
        self.apf_seats = 0
        self.apf_queue = 50
        self.apf_queue_wait_s = 15.0
        self.service_ms = 0.0
        self.read_service_ms = 0.0
        self.h2: dict = {}  # HTTP/2 connections opened from now on: h2_max_streams, h2_goaway_after (h2.py)

    def match(self, method: str, plural: str, name: str | None) -> tuple | None:
        """(error, after) of the targeted rule this request matches, or None.  `after`: the request is
        served and *then* answered with the error (a lost response, or a concurrent writer that won the
        race: the object changed, the client is told it conflicted)."""
        for r in self.rules:
            if r.get("count", -1) == 0:
                continue
            if r.get("method", "*") not in ("*", method) or r.get("resource", "*") not in ("*", plural) or \
                    r.get("name", "*") not in ("*", name):
                continue
            if r.get("count", -1) > 0:
                r["count"] -= 1
            err = E.from_status(int(r.get("code", 500)), {"reason": r.get("reason", ""),
                                                          "message": r.get("message", "injected fault")})
            if r.get("retry_after") is not None:  # answered with a Retry-After header
                err.retry_after = float(r["retry_after"])
            return err, bool(r.get("after"))
        return None

    def update(self, d: dict) -> None:
        if "rules" in d:
            self.rules = [dict(r) for r in d["rules"] or ()]
        for k in ("latency_ms", "jitter_ms", "error_rate", "throttle_rate", "apf_queue_wait_s", "service_ms",
                  "read_service_ms"):
            if k in d:
                setattr(self, k, float(d[k]))
        for k in ("max_mutating_inflight", "apf_seats", "apf_queue"):
            if k in d:
                setattr(self, k, int(d[k]))
        if "error_code" in d:
            self.error_code = int(d["error_code"])
        if "down" in d:
            self.down = bool(d["down"])
        if "write_only" in d:
            self.write_only = bool(d["write_only"])
        for k in ("h2_max_streams", "h2_goaway_after", "h2_initial_window", "h2_small_conn_window"):
            if k in d:
                self.h2[k] = int(d[k])

    def as_dict(self) -> dict:
        return dict(self.__dict__)


class FakeApiServer:
    def __init__(self, state: ClusterState | None = None, *, name: str = "fake", token: str | None = None,
                 bookmark_interval: float = 5.0, crd_dir: str | None = None, http2: bool = True):
        self.state = state or ClusterState(name)
        if crd_dir:  # validate custom-resource writes against these CRDs' schemas (422 Invalid)
            from ..api.schema import load_crds
            self.state.crds.update(load_crds(crd_dir))
        self._routes: dict = {}  # path -> parsed route (see _parse)
        self.name = name
        self.token = token
        self.bookmark_interval = bookmark_interval
        self.faults = Faults()
        self.flow = FlowControl()
        self.markers = MarkerTracker()
        self.staged: dict[str, dict] = {}  # /_fake/stage: pre-decoded apply bodies by id
        self.state.write_hooks.append(self.markers.on_write)
        self.requests = {"total": 0, "watch_streams": 0, "errors_injected": 0, "throttled": 0}
        # (method, plural, name, subresource, status) of every mutating request (tests count writes per object)
        self.writes: list[tuple] = []
        self.record_writes = False  # in-process test servers turn it on (FakeEnvironment)
        self._streams: set = set()
        self._http = web.HttpServer(self._dispatch, fast=self.fast)
        # HTTP/2 as a kube-apiserver serves it: ALPN "h2" on TLS, and prior knowledge on cleartext (ncc/fakeapi/h2.py)
        self._http.http2 = http2
        self._http.h2_options = self.faults.h2
        self.port: int | None = None
        self.url: str | None = None

    # ------------------------------------------------------------------ lifecycle
    async def start(self, host: str = "127.0.0.1", port: int = 0, ssl_context: ssl.SSLContext | None = None) -> str:
        if ssl_context is not None and self._http.http2:
            ssl_context.set_alpn_protocols(["h2", "http/1.1"])
        self.port = await self._http.start(host, port, ssl_context)
        self.url = f"{'https' if ssl_context else 'http'}://{host}:{self.port}"
        return self.url

    async def stop(self) -> None:
        self.state.close_watchers()
        await self._http.stop()

    WATCH_COALESCE_S = 0.0005  # see _watch

    def drop_watches(self) -> None:
        self.state.close_watchers()

    # ------------------------------------------------------------------ routing
    def _parse(self, path: str):
        """→ (rt, namespace, name, subresource) or a special-route string; memoised per path (writes
        repeat the same object paths wave after wave)."""
        hit = self._routes.get(path)
        if hit is not None:
            return hit
        out = self._parse_uncached(path)
        if len(self._routes) > 65536:
            self._routes.clear()
        self._routes[path] = out
        return out

    def _parse_uncached(self, path: str):
        parts = [p for p in path.split("/") if p]
        if not parts:
            return "root"
        if parts[0] == "api":
            if len(parts) == 1:
                return "api"
            group, version, rest = "", parts[1], parts[2:]
        elif parts[0] == "apis":
            if len(parts) == 1:
                return "apis"
            if len(parts) < 3:
                return "apigroup"
            group, version, rest = parts[1], parts[2], parts[3:]
        else:
            return "/".join(parts)
        if not rest:
            return ("resources", group, version)
        ns = None
        if rest[0] == "namespaces" and len(rest) >= 3:
            ns, rest = rest[1], rest[2:]
        elif rest[0] == "namespaces" and len(rest) <= 2:
            rt = self.state.resource("", "namespaces")
            return rt, None, (rest[1] if len(rest) == 2 else None), None
        plural = rest[0]
        name = rest[1] if len(rest) > 1 else None
        sub = rest[2] if len(rest) > 2 else None
        rt = self.state.resource(group, plural)
        if rt.version != version:
            raise E.NotFound(f"version {version} of {plural}.{group} not served")
        return rt, ns, name, sub

    def fast(self, request: web.Request):
        """Synchronous handling of plain CRUD requests — no task, no await — used by the HTTP layer for
        every request that is not a control endpoint, a watch, or subject to injected latency."""
        if request.path.startswith("/_fake/"):
            return None
        f = self.faults
        if f.latency_ms or f.jitter_ms:
            return None
        if request.method == "GET" and "watch=" in request.raw_query:
            return None
        self.requests["total"] += 1
        if FlowControl.active(f) and not f.down and request.path.startswith(("/api/", "/apis/")):
            return self._admitted(request)
        return self._core(request)

    def _admitted(self, request: web.Request):
        """Serve a request through the admission model (flowcontrol.py): a 429 at once, or a Deferred answered
        once it held a seat for its service time."""
        f = self.faults
        mutating = request.method in ("POST", "PUT", "PATCH", "DELETE")
        d = web.Deferred()

        def run():
            try:
                resp = self._core(request)
            except Exception as e:  # noqa: BLE001
                resp = web.Response(500, text=f"internal error: {e}")
            finally:
                self.flow.release(mutating)
            d.resolve(resp)

        def granted(err=None):
            if err is not None:  # its wait for a seat ran out
                self.requests["throttled"] += 1
                d.resolve(_status_response(err))
                return
            delay = FlowControl.service_s(f, mutating)
            if delay > 0:
                asyncio.get_running_loop().call_later(delay, run)
            else:
                run()
        err = self.flow.admit(f, mutating, granted)
        if err is not None:
            self.requests["throttled"] += 1
            return _status_response(err)
        return d

    async def _dispatch(self, request: web.Request) -> web.StreamResponse:
        self.requests["total"] += 1
        path = request.path
        if path.startswith("/_fake/"):
            return await self._control(request, path[len("/_fake/"):])
        f = self.faults
        api = path.startswith(("/api/", "/apis/"))
        if (f.latency_ms or f.jitter_ms) and api and not f.down:
            await asyncio.sleep((f.latency_ms + random.random() * f.jitter_ms) / 1000.0)
        if api and FlowControl.active(f) and not f.down and \
                not (request.method == "GET" and "watch=" in request.raw_query):
            d = self._admitted(request)
            if not isinstance(d, web.Deferred):
                return d
            if d.response is None:
                fut = asyncio.get_running_loop().create_future()
                d.then(fut.set_result)
                return await fut
            return d.response
        r = self._core(request)
        if isinstance(r, tuple):  # a watch
            return await self._watch(request, r[1], r[2])
        return r

    def _core(self, request: web.Request):
        """`_serve` plus the write log."""
        r = self._serve(request)
        if self.record_writes and request.method in ("POST", "PUT", "PATCH", "DELETE") and \
                not isinstance(r, tuple) and request.path.startswith(("/api/", "/apis/")):
            target = self._routes.get(request.path)
            if isinstance(target, tuple) and len(target) == 4:
                self.writes.append((request.method, target[0].plural, target[2], target[3], r.status,
                                    time.monotonic()))
                if len(self.writes) > 100000:
                    del self.writes[:50000]
        return r

    def _serve(self, request: web.Request):
        """Auth, faults, routing and CRUD for one request; returns a Response, or ("watch", rt, ns)."""
        path = request.path
        if path in ("/healthz", "/readyz", "/livez"):
            return web.Response(text="ok")
        if path == "/version":
            return web.Response(body=_dumps({"major": "1", "minor": "33", "gitVersion": "v1.33.0-ncc-fake",
                                             "platform": "linux/amd64"}), content_type=_JSON)
        try:
            if self.token is not None:
                auth = request.headers.get("authorization", "")
                if auth != f"Bearer {self.token}":
                    raise E.Unauthorized("Unauthorized")
            f = self.faults
            if f.down:
                raise E.ServiceUnavailable("the server is currently unable to handle the request")
            mutating = request.method in ("POST", "PUT", "PATCH", "DELETE")
            if f.throttle_rate and random.random() < f.throttle_rate:
                self.requests["throttled"] += 1
                raise E.TooManyRequests("too many requests, please try again later", retry_after=1)
            if f.error_rate and (mutating or not f.write_only) and random.random() < f.error_rate:
                self.requests["errors_injected"] += 1
                raise E.from_status(f.error_code, {"message": "injected fault"})
            target = self._parse(path)
            if isinstance(target, str):
                return self._discovery(target)
            if target[0] == "resources":
                return self._resource_list(target[1], target[2])
            rt, ns, name, sub = target
            m = request.method
            if f.rules:
                if m == "POST" and name is None:  # a create names its object in the body
                    name = ((self._body(request) or {}).get("metadata") or {}).get("name")
                hit = f.match(m, rt.plural, name)
                if hit is not None:
                    self.requests["errors_injected"] += 1
                    if not hit[1]:
                        raise hit[0]
                    self._crud(request, path, rt, ns, target[2], sub)  # served, then answered with the error
                    raise hit[0]
            return self._crud(request, path, rt, ns, target[2], sub)
        except E.ApiError as e:
            return _status_response(e)
        except (ValueError, KeyError, TypeError) as e:
            return _status_response(E.BadRequest(f"bad request: {e}"))

    def _crud(self, request: web.Request, path: str, rt, ns, name, sub):
        q = request.query
        m = request.method
        if m == "GET":
            if name is None:
                if q.get("watch") in ("1", "true"):
                    return ("watch", rt, ns)
                limit = int(q["limit"]) if q.get("limit") else None
                return self._json(self.state.list(rt, ns, label_selector=q.get("labelSelector"), limit=limit,
                                                  continue_token=q.get("continue")))
            return self._json(self.state.get(rt, ns or "", name))
        body = self._body(request) if m != "DELETE" or request.can_read_body else None
        if m == "POST" and name is None:
            return self._written(self.state.create(rt, ns or "", body, owned=True), 201)
        if m == "PUT" and name is not None:
            if (body.get("metadata") or {}).get("name") not in (None, name):
                raise E.BadRequest("the name of the object does not match the name on the URL")
            body.setdefault("metadata", {})["name"] = name
            if sub not in (None, "status"):
                raise E.NotFound(f"subresource {sub} not found")
            if sub == "status" and not rt.has_status:
                raise E.NotFound(f"{rt.plural} has no status subresource")
            return self._written(self.state.update(rt, ns or "", body, subresource=sub, owned=True))
        if m == "PATCH" and name is not None:
            ctype = request.content_type
            if ctype not in (PATCH_MERGE, PATCH_STRATEGIC, PATCH_JSON, PATCH_APPLY):
                raise E.ApiError(f"unsupported patch type {ctype}", code=415, reason="UnsupportedMediaType")
            return self._written(self.state.patch(rt, ns or "", name, body, ctype, subresource=sub,
                                                  manager=q.get("fieldManager", "")))
        if m == "DELETE" and name is not None:
            opts = body or {}
            return self._json(self.state.delete(rt, ns or "", name, preconditions=opts.get("preconditions"),
                                                propagation_policy=opts.get("propagationPolicy")
                                                or q.get("propagationPolicy")))
        raise E.MethodNotAllowed(f"method {m} not allowed on {path}")

    @staticmethod
    def _body(request: web.Request):
        raw = request.body
        if not raw:
            return {}
        if request.content_type == PATCH_APPLY:
            try:
                return loads_bytes(raw)
            except ValueError:
                import yaml
                return yaml.safe_load(raw)
        return loads_bytes(raw)

    @staticmethod
    def _json(obj, status: int = 200) -> web.Response:
        return web.Response(status=status, body=_dumps(obj), content_type=_JSON)

    def _written(self, obj, status: int = 200) -> web.Response:
        """Write response; reuses the watch event's encoding of the same object when there is one."""
        body = self.state.encoded(obj)
        return web.Response(status=status, body=body if body is not None else _dumps(obj), content_type=_JSON)

    # ------------------------------------------------------------------ discovery
    def _discovery(self, target: str) -> web.Response:
        if target == "api":
            return self._json({"kind": "APIVersions", "versions": ["v1"]})
        if target == "apis":
            groups = sorted({(g, v) for (g, _p), rt in self.state._types.items() if g for v in [rt.version]})
            return self._json({"kind": "APIGroupList", "apiVersion": "v1", "groups": [
                {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v}],
                 "preferredVersion": {"groupVersion": f"{g}/{v}", "version": v}} for g, v in groups]})
        if target == "root":
            return self._json({"paths": ["/api", "/apis", "/healthz", "/version"]})
        raise E.NotFound(f"the server could not find the requested resource {target}")

    def _resource_list(self, group: str, version: str) -> web.Response:
        res = []
        for (g, plural), rt in sorted(self.state._types.items()):
            if g == group and rt.version == version:
                res.append({"name": plural, "namespaced": rt.namespaced, "kind": rt.kind,
                            "verbs": ["create", "delete", "get", "list", "patch", "update", "watch"]})
                if rt.has_status:
                    res.append({"name": f"{plural}/status", "namespaced": rt.namespaced, "kind": rt.kind,
                                "verbs": ["get", "patch", "update"]})
        gv = f"{group}/{version}" if group else version
        return self._json({"kind": "APIResourceList", "apiVersion": "v1", "groupVersion": gv, "resources": res})

    # ------------------------------------------------------------------ watch
    async def _watch(self, request: web.Request, rt: R.ResourceType, ns: str | None) -> web.StreamResponse:
        q = request.query
        timeout = float(q["timeoutSeconds"]) if q.get("timeoutSeconds") else None
        bookmarks = q.get("allowWatchBookmarks") in ("1", "true")
        try:
            w = self.state.watch(rt, ns, q.get("resourceVersion"), q.get("labelSelector"))
        except E.Gone as e:
            # like the apiserver: an in-stream ERROR event carrying a 410 Status
            resp = web.StreamResponse(status=200, headers={"Content-Type": _JSON})
            await resp.prepare(request)
            await resp.write(_dumps({"type": "ERROR", "object": e.status_object()}) + b"\n")
            await resp.write_eof()
            return resp
        resp = web.StreamResponse(status=200, headers={"Content-Type": _JSON})
        await resp.prepare(request)
        self.requests["watch_streams"] += 1
        self._streams.add(w)
        loop = asyncio.get_running_loop()
        deadline = loop.time() + timeout if timeout else None
        last_bookmark = loop.time()
        last_write = 0.0
        try:
            while True:
                now = loop.time()
                wait = self.bookmark_interval if bookmarks else 3600.0
                if deadline is not None:
                    wait = min(wait, deadline - now)
                    if wait <= 0:
                        break
                if not w.queue.empty():
                    rec = w.queue.get_nowait()
                else:
                    try:
                        rec = await wait_timeout(w.queue.get(), max(wait, 0.0))
                    except asyncio.TimeoutError:
                        rec = False
                if rec is None:
                    break
                if rec is not False and loop.time() - last_write < self.WATCH_COALESCE_S:
                    # under sustained load, let a few more events join this write (one syscall and one
                    # consumer wake-up per batch instead of per event); an isolated event goes out at once
                    await asyncio.sleep(self.WATCH_COALESCE_S)
                chunks = []
                if rec is not False:
                    chunks.append(rec.line())
                    while not w.queue.empty():  # batch everything already queued into one write
                        nxt = w.queue.get_nowait()
                        if nxt is None:
                            rec = None
                            break
                        chunks.append(nxt.line())
                if bookmarks and loop.time() - last_bookmark >= self.bookmark_interval:
                    chunks.append(_dumps({"type": "BOOKMARK", "object": {
                        "kind": rt.kind, "apiVersion": rt.api_version,
                        "metadata": {"resourceVersion": str(self.state.rv)}}}) + b"\n")
                    last_bookmark = loop.time()
                if chunks:
                    await resp.write(b"".join(chunks))
                    last_write = loop.time()
                if rec is None:
                    break
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            w.close()
            self._streams.discard(w)
        try:
            await resp.write_eof()
        except (ConnectionResetError, RuntimeError):
            pass
        return resp

    # ------------------------------------------------------------------ control
    async def _control(self, request: web.Request, what: str) -> web.Response:
        if what == "stats":
            counts = {f"{g or 'core'}/{p}": self.state.count(rt) for (g, p), rt in self.state._types.items()}
            return self._json({"name": self.name, "rv": self.state.rv, "requests": self.requests,
                               "state": self.state.stats, "objects": counts, "faults": self.faults.as_dict(),
                               "admission": self.state.admission.as_dict(),
                               "watchers": len(self.state._watchers), "connections": self._http.conn_stats(),
                               "flow": self.flow.stats()})
        if what == "writes":
            return self._json({"writes": [list(w) for w in self.writes]})
        if what == "faults" and request.method == "POST":
            body = self._body(request)
            self.faults.update(body)
            if "record_writes" in body:  # a subprocess server's write log (GET /_fake/writes), on demand
                self.record_writes = bool(body["record_writes"])
                self.writes.clear()
            if body.get("compact") or body.get("relist"):
                # compaction first: a client whose watch is dropped next must find its revision gone
                self.state.compact(advance=bool(body.get("relist")))
            if body.get("drop_watches") or body.get("down") or body.get("relist"):
                self.drop_watches()
            return self._json(self.faults.as_dict())
        if what == "admission" and request.method == "POST":
            self.state.admission.update(self._body(request))
            return self._json(self.state.admission.as_dict())
        if what == "markers" and request.method == "POST":
            body = self._body(request)
            for plural, path in (body.get("specs") or {}).items():
                self.markers.add_spec(plural, path)
            return self._json({"specs": {k: ".".join(v) for k, v in self.markers.paths.items()}})
        if what == "markers/wait" and request.method == "POST":
            body = self._body(request)
            want = body.get("want") or []
            ok = await self.markers.wait(want, float(body.get("timeout", 60)))
            out = {"ok": ok, "counts": {f"{w['plural']}={w['value']}": len(self.markers.times(w["plural"], w["value"]))
                                        for w in want}}
            if body.get("times"):
                keyed = bool(body.get("keyed"))
                out["times"] = {f"{w['plural']}={w['value']}": self.markers.times(w["plural"], w["value"], keyed)
                                for w in want}
            return self._json(out)
        if what == "stage" and request.method == "POST":
            # a load generator's apply body, decoded ahead of time and committed later by
            # {"staged": id} — so a timed apply measures commits, not the decoding of the request
            body = self._body(request)
            self.staged[str(body["id"])] = body
            return self._json({"staged": str(body["id"]), "items": len(body.get("items") or [])})
        if what == "apply" and request.method == "POST":
            body = self._body(request)
            if "staged" in body:
                body = self.staged.pop(str(body["staged"]))
            t0 = time.time_ns()
            n = 0
            # yield_every > 0 lets watch streams flush while a large apply is in progress (commits and
            # watch delivery interleave, as on a real apiserver serving many concurrent writers)
            yield_every = int(body.get("yield_every") or 0)
            for o in body.get("items") or []:
                if yield_every and n and n % yield_every == 0:
                    await asyncio.sleep(0)
                rt = R.by_kind(o["kind"])
                m = o.get("metadata") or {}
                ns = m.get("namespace", "")
                try:
                    cur = self.state.get(rt, ns, m["name"])
                except E.NotFound:
                    cur = None
                if cur is None:
                    self.state.create(rt, ns, o, owned=True)
                else:
                    new = dict(cur)
                    for k, v in o.items():
                        if k not in ("metadata", "status", "apiVersion", "kind"):
                            new[k] = v
                    new["metadata"] = dict(cur["metadata"])
                    for mk in ("labels", "annotations"):
                        if mk in m:
                            new["metadata"][mk] = m[mk]
                    self.state.update(rt, ns, new, owned=True)
                n += 1
            return self._json({"applied": n, "t0_ns": t0, "t1_ns": time.time_ns(), "rv": self.state.rv})
        if what == "objects" and request.method == "POST":
            body = self._body(request)
            n = 0
            for o in body.get("items") or []:
                rt = R.by_kind(o["kind"])
                owner = o.pop("__owner_template__", None)
                if owner:  # seed a dependent owned by an existing template (resolve its live UID)
                    ns_ = (o.get("metadata") or {}).get("namespace", "")
                    t = self.state.get(R.TEMPLATES, ns_, owner)
                    o.setdefault("metadata", {})["ownerReferences"] = [{
                        "apiVersion": t["apiVersion"], "kind": t["kind"], "name": owner,
                        "uid": t["metadata"]["uid"]}]
                try:
                    self.state.create(rt, (o.get("metadata") or {}).get("namespace", ""), o)
                    n += 1
                except E.AlreadyExists:
                    pass
            return self._json({"created": n, "rv": self.state.rv})
        return web.Response(status=404, text="unknown control endpoint")


async def serve(args) -> None:
    logging.basicConfig(level=logging.WARNING)
    server = FakeApiServer(name=args.name, token=args.token, bookmark_interval=args.bookmark_interval,
                           crd_dir=args.crd_dir, http2=not getattr(args, "no_http2", False))
    for m in args.marker:
        plural, _, path = m.partition("=")
        server.markers.add_spec(plural, path)
    sets: dict = {}
    for a in args.admission_set:  # plural=dotted.path=<json value>
        plural, _, rest = a.partition("=")
        path, _, value = rest.partition("=")
        sets.setdefault(plural, {})[path] = json.loads(value)
    server.state.admission.update({"prune_defaults": args.prune_defaults, "sets": sets})
    ctx = None
    if args.tls_cert:
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(args.tls_cert, args.tls_key)
        if args.tls_client_ca:  # x509 client auth (kube-apiserver --client-ca-file)
            ctx.load_verify_locations(cafile=args.tls_client_ca)
            ctx.verify_mode = ssl.CERT_REQUIRED
    url = await server.start(args.host, args.port, ctx)
    from .. import gctune
    gctune.collect_startup()  # before it serves anyone
    gctune.tune(account=False)
    # A test server that keeps what it allocates: freeze every second, never scan the survivors (gctune);
    # NCC_FAKEAPI_GC=collect restores the round-2 controller policy (generation-1 pass + freeze every 5 s)
    if os.environ.get("NCC_FAKEAPI_GC") == "collect":
        gc_task = asyncio.ensure_future(gctune.freeze_loop(5.0, collect=1, full_period=0))
    else:
        gc_task = asyncio.ensure_future(gctune.freeze_loop(1.0, full_period=0, young=False))
    from .. import loopmon
    lag_task = loopmon.start(f"fakeapi:{args.name}")
    if args.port_file:
        tmp = args.port_file + ".tmp"
        with open(tmp, "w") as f:
            f.write(url)
        os.replace(tmp, args.port_file)
    print(url, flush=True)
    stop = asyncio.Event()
    loop = asyncio.get_running_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        loop.add_signal_handler(sig, stop.set)
    if args.parent_pid:
        async def watch_parent():
            while True:
                await asyncio.sleep(1.0)
                try:
                    os.kill(args.parent_pid, 0)
                except OSError:
                    stop.set()
                    return
        asyncio.ensure_future(watch_parent())
    await stop.wait()
    gc_task.cancel()
    if lag_task is not None:
        lag_task.cancel()
    await server.stop()


def main(argv=None) -> None:
    from ..proclimits import raise_nofile_limit
    raise_nofile_limit()
    p = argparse.ArgumentParser(prog="python -m ncc.fakeapi", description="in-process fake kube-apiserver")
    p.add_argument("--name", default="fake")
    p.add_argument("--host", default="127.0.0.1")
    p.add_argument("--port", type=int, default=0)
    p.add_argument("--port-file")
    p.add_argument("--token")
    p.add_argument("--tls-cert")
    p.add_argument("--tls-key")
    p.add_argument("--tls-client-ca", help="require client certificates signed by this CA (mutual TLS)")
    p.add_argument("--crd-dir", help="validate custom-resource writes against the CRDs in this directory")
    p.add_argument("--prune-defaults", action="store_true",
                   help="apply the --crd-dir schemas' defaults and prune unknown fields on writes (as an apiserver)")
    p.add_argument("--admission-set", action="append", default=[], metavar="PLURAL=PATH=JSON",
                   help="mutating-webhook stand-in: write this field into every create/update (repeatable)")
    p.add_argument("--bookmark-interval", type=float, default=5.0)
    p.add_argument("--no-http2", action="store_true",
                   help="HTTP/1.1 only: no ALPN h2 on TLS, no prior-knowledge HTTP/2 on cleartext")
    p.add_argument("--parent-pid", type=int, default=0, help="exit when this process disappears")
    p.add_argument("--marker", action="append", default=[], help="plural=field.path propagation probe (repeatable)")
    args = p.parse_args(argv)
    prof_path = os.environ.get("NCC_FAKEAPI_PROFILE")
    if prof_path:  # NCC_FAKEAPI_PROFILE=/path/prefix → /path/prefix.<name>
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
        try:
            asyncio.run(serve(args))
        finally:
            prof.disable()
            prof.dump_stats(f"{prof_path}.{args.name}")
        return
    asyncio.run(serve(args))


if __name__ == "__main__":
    main()
