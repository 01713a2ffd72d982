"""Coordinator-side support for the native shard executor (`ncc/bin/ncc-executor`, native/executor/).

The C++ executor is a drop-in for the Python executor process (`python -m ncc.executor`): same
supervision (`ExecutorHandle`), same socketpair protocol, same reports.  It never talks to the
controller cluster — the coordinator's watch relay feeds it (ncc/controller/relay.py) — so the
coordinator hands it everything else it needs as the first message on the channel:

    {"t": "cfg", "c": "<json>"}   options + per-shard connection details with *resolved* credentials

Kubeconfig parsing, `tokenFile` paths and `exec` credential plugins (EKS `aws eks get-token`) stay in
Python (ncc/kube/kubeconfig.py): the executor receives the server URL, CA / client certificate PEMs,
and a bearer token; exec tokens are refreshed here and pushed as `{"t": "cred"}` messages.

`executor-impl: auto` (default) picks the native executor whenever the binary is built and the
configuration is one it implements (native mode with the watch relay; POST/PUT writes, or server-side
apply with `server-side-apply: true`); otherwise the Python executor runs — loudly: a Warning at start-up,
the `executor_native` gauge at 0, and `/readyz?verbose` and `/debug/state` name the reason (ncc/app.py).

Why three implementations of the reconcile semantics — the in-process one
(ncc/controller/reconcile.py: compat mode and the reference's own test harness), the Python executor and the
C++ executor — and not two: the Python executor is what `pip install` gives a host without a C++20 compiler or
libssl headers (setup.py builds the executor best-effort), and what runs with `watch-relay: false`; and it is
the readable specification the C++ executor is conformance-tested against, scenario by scenario
(tests/test_conformance.py runs every scenario on "inprocess", "python" and "native").  The container image
requires the C++ executor (NCC_REQUIRE_EXECUTOR=1 at build, NCC_REQUIRE_NATIVE=1 at run).
"""
from __future__ import annotations

import asyncio
import json
import logging
import os

from ..kube.kubeconfig import CredentialSource, load_kubeconfig
from ..shards.loader import discover

log = logging.getLogger("ncc.executor")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# keep-alive connections per shard, and pipelined requests on each, when `client-pool-size` /
# `client-pipeline-depth` are 0 (auto): 256 requests in flight at most.  No pipelining by default: an
# HTTP/1.1 server (kube-apiserver's Go net/http) serves one connection's requests one after the other, so
# only connections give a shard apiserver requests to run concurrently (APF seats, etcd round trips); and on
# the bench, 32 connections × 8 coalesced only 1.3 requests per write (docs/BENCHMARKS_ARCHIVE.md).  Pipelining pays for a
# far-away shard, where the round trip rather than the apiserver bounds a connection.  256 is also the HTTP/1.1
# connection count, and a kube-apiserver admits 200 mutating requests at a time by default.
DEFAULT_POOL_SIZE = 256
DEFAULT_PIPELINE_DEPTH = 1
# Over HTTP/2 a request in flight is a stream, not a connection: with client-pool-size auto, a shard that speaks
# HTTP/2 may have this many in flight (the adaptive limit still starts at 128 and backs off on 429s), so a shard
# milliseconds away is not bound by 256 ÷ RTT (BENCHMARKS.md "Shards × round-trip latency": 1024 in flight gave
# +35 % at 5 ms and +121 % at 20 ms).  An explicit client-pool-size caps both protocols; a shard that falls back to
# HTTP/1.1 gets pool × depth again (http.hpp `Client::h2_off`).
DEFAULT_H2_INFLIGHT = 1024
_LEVELS = {"DEBUG": 10, "INFO": 20, "WARNING": 30, "WARN": 30, "ERROR": 40, "CRITICAL": 50}


def binary_path() -> str | None:
    p = os.environ.get("NCC_EXECUTOR_BINARY") or os.path.join(ROOT, "ncc", "bin", "ncc-executor")
    return p if os.path.isfile(p) and os.access(p, os.X_OK) else None


def choose(cfg, options, relay_active: bool, quiet: bool = False) -> tuple[bool, str]:
    """(use the native executor?, why not).  `relay_active`: the coordinator's watch relay feeds the
    executors (a precondition: the native executor has no controller-cluster client)."""
    # NCC_EXECUTOR_IMPL overrides the config (lets a test run / CI job pin either implementation)
    impl = (os.environ.get("NCC_EXECUTOR_IMPL") or cfg.executor_impl or "auto").lower()
    if impl == "python":
        return False, "executor-impl: python"
    reasons = []
    if binary_path() is None:
        reasons.append("ncc/bin/ncc-executor is not built (python native/build.py)")
    if not relay_active:
        reasons.append("the watch relay is off")
    if reasons:
        if impl == "native" and not quiet:
            log.warning("executor-impl: native requested but unavailable (%s); using the Python executor",
                        "; ".join(reasons))
        return False, "; ".join(reasons)
    return True, ""


def _file_digest(path: str) -> str:
    import hashlib
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()
    except OSError:
        return ""


def proxy_entry(cc) -> dict:
    """The shard's proxy for the C++ executor: its URL and the CONNECT request (credentials included), rendered
    here so the executor needs no URL or base64 handling of its own (ncc/kube/proxy.py)."""
    from urllib.parse import unquote, urlsplit

    from ..kube.proxy import connect_request, proxy_for
    proxy = proxy_for(cc.server, cc.proxy_url)
    if not proxy:
        return {}
    u, p = urlsplit(cc.server), urlsplit(proxy)
    phost = f"[{p.hostname}]" if p.hostname and ":" in p.hostname else (p.hostname or "")
    if p.scheme in ("socks5", "socks5h"):  # the executor runs the SOCKS5 handshake itself (http.hpp Conn::connect)
        return {"proxy": f"socks5://{phost}:{p.port or 1080}",
                "proxy_user": unquote(p.username) if p.username is not None else "",
                "proxy_pass": unquote(p.password or "")}
    # the credentials travel in the rendered request only
    return {"proxy": f"http://{phost}:{p.port or 80}",
            "proxy_connect": connect_request(proxy, u.hostname or "",
                                             u.port or (443 if u.scheme == "https" else 80)).decode()}


class NativeExecutorConfig:
    """Renders the `cfg` message of one executor and keeps exec-plugin tokens fresh."""

    def __init__(self, cfg, options):
        self.cfg = cfg
        self.options = options
        self.paths = dict(discover(cfg.shard_config_path))
        self.creds: dict[str, CredentialSource] = {}
        self.tokens: dict[str, str | None] = {}
        self.digests: dict[str, str] = {}  # sha256 of the kubeconfig each cached CredentialSource came from

    def _source(self, name: str) -> CredentialSource:
        """The shard's credentials, re-read when its kubeconfig file changed since they were loaded (a rotated
        CA, server or client certificate must reach the next executor spawned for it)."""
        self.paths = dict(discover(self.cfg.shard_config_path))
        path = self.paths[name]
        digest = _file_digest(path)
        src = self.creds.get(name)
        if src is None or self.digests.get(name) != digest:
            cc = load_kubeconfig(path, name=name)
            src = self.creds[name] = CredentialSource(cc)
            self.digests[name] = digest
            self.tokens.pop(name, None)
        return src

    def forget(self, names) -> None:
        """Drop what is cached for shards that were removed or changed (App.reload_shards): their next
        executor re-reads the kubeconfig, and the token refresher stops serving removed shards."""
        for n in names:
            self.creds.pop(n, None)
            self.tokens.pop(n, None)
            self.digests.pop(n, None)

    async def shard_entry(self, name: str) -> dict:
        src = self._source(name)
        cc = src.cfg
        token = await src.token() if (cc.exec is not None or cc.token) else None
        self.tokens[name] = token
        cert, key = cc.client_cert_data, cc.client_key_data
        exec_cert = await src.exec_client_cert()
        if exec_cert:
            cert, key = exec_cert
        return {"name": name, "server": cc.server, "ca_pem": (cc.ca_data or b"").decode(), "insecure": cc.insecure,
                "tls_server_name": cc.tls_server_name or "", "cert_pem": (cert or b"").decode(),
                "key_pem": (key or b"").decode(), "token": token or "",
                "token_file": cc.token_file if (cc.token_file and not cc.token and cc.exec is None) else "",
                "username": cc.username or "", "password": cc.password or "", **proxy_entry(cc)}

    async def render(self, handle) -> str:
        from ..app import client_limits
        from ..config import HTTP2_MODES
        o, cfg = self.options, self.cfg
        shards = [await self.shard_entry(n) for n in handle.shards]
        qps, burst = client_limits(cfg)
        pool = cfg.client_pool_size if cfg.client_pool_size > 0 else DEFAULT_POOL_SIZE
        depth = cfg.client_pipeline_depth if cfg.client_pipeline_depth > 0 else DEFAULT_PIPELINE_DEPTH
        doc = {
            "namespace": cfg.controller_namespace, "alias": cfg.alias,
            # one C++ process per shard carries all of its concurrency: like client-go's HTTP/2 connection
            # (up to 250 concurrent streams) up to pool × depth requests in flight per shard, pipelined on
            # `pool` keep-alive connections, under an adaptive limit (http.hpp `Client`: slow start, AIMD on
            # 429/503/timeouts) and the client-qps bucket
            "workers": 4 * max(DEFAULT_POOL_SIZE * DEFAULT_PIPELINE_DEPTH, pool * depth), "pool_size": pool,
            "pipeline_depth": depth, "client_qps": qps, "client_burst": burst,
            "h2_inflight": DEFAULT_H2_INFLIGHT if cfg.client_pool_size <= 0 else 0,
            "http2": HTTP2_MODES.get(str(cfg.client_http2).lower(), 1),
            "request_timeout": 30.0, "coalesce_window": o.coalesce_window,
            "failure_base_delay": o.failure_base_delay, "failure_max_delay": o.failure_max_delay,
            "rate_limit_qps": o.rate_limit_qps, "rate_limit_burst": o.rate_limit_burst,
            "shard_sync_timeout": o.wait_for_shards_timeout if o.wait_for_shards_timeout is not None else 3600.0,
            "full_resync_period": o.full_resync_period, "sync_binary_data": o.sync_binary_data,
            "sync_secret_type": o.sync_secret_type, "orphan_sweep": o.orphan_sweep,
            "propagate_workgroup_deletes": o.propagate_workgroup_deletes, "server_side_apply": o.server_side_apply,
            "sync_dependent_metadata": o.sync_dependent_metadata,
            "log_level": _LEVELS.get(str(cfg.log_level).upper(), 30), "shards": shards,
        }
        return json.dumps(doc)

    async def refresh_loop(self, pool, period: float = 30.0) -> None:
        """Push rotated exec-plugin tokens to the executors serving each shard."""
        while True:
            await asyncio.sleep(period)
            for name, src in list(self.creds.items()):
                if src.cfg.exec is None:
                    continue
                try:
                    tok = await src.token()
                except Exception as e:  # noqa: BLE001
                    log.warning("refreshing the credential of shard %s: %s", name, e)
                    continue
                if tok and tok != self.tokens.get(name):
                    self.tokens[name] = tok
                    for h in pool.handles:
                        if h.native and name in h.shards and h.channel is not None:
                            h.channel.send({"t": "cred", "s": name, "token": tok})
