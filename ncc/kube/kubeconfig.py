"""kubeconfig / in-cluster configuration loading (client-go `clientcmd` + `rest.InClusterConfig` subset).

The reference builds the controller-cluster config with
`clientcmd.BuildConfigFromFlags("", ControllerConfigPath)` (main.go:52) — an empty path means
in-cluster — and one config per shard from `<shard>.kubeconfig` files (README.md:15-28).
Shards on EKS authenticate through the kubeconfig `exec` plugin (`aws eks get-token`), which is
why the reference image bundles the AWS CLI (.container/Dockerfile:16-41).

Supported: current-context / explicit context, `server`, `certificate-authority(-data)`,
`insecure-skip-tls-verify`, `tls-server-name`, `proxy-url` (an HTTP CONNECT proxy; without it, client-go's
`HTTPS_PROXY`/`HTTP_PROXY`/`NO_PROXY`, `ncc/kube/proxy.py`), `client-certificate(-data)`/`client-key(-data)`,
`token`/`tokenFile`, basic auth, and `exec` credential plugins
(client.authentication.k8s.io/v1 and v1beta1) with expiry-aware caching.
"""
from __future__ import annotations

import asyncio
import base64
import datetime as _dt
import json
import os
import time
from dataclasses import dataclass, field

import yaml

SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"


class ConfigError(Exception):
    pass


@dataclass
class ExecConfig:
    command: str
    args: list = field(default_factory=list)
    env: list = field(default_factory=list)  # [{"name":..,"value":..}]
    api_version: str = "client.authentication.k8s.io/v1"
    provide_cluster_info: bool = False
    interactive_mode: str = "Never"


@dataclass
class ClusterConfig:
    server: str
    name: str = ""
    ca_data: bytes | None = None
    insecure: bool = False
    tls_server_name: str | None = None
    client_cert_data: bytes | None = None
    client_key_data: bytes | None = None
    token: str | None = None
    token_file: str | None = None
    username: str | None = None
    password: str | None = None
    exec: ExecConfig | None = None
    namespace: str | None = None
    base_dir: str = ""
    proxy_url: str | None = None  # kubeconfig `proxy-url`

    @property
    def is_tls(self) -> bool:
        return self.server.startswith("https://")


def _read(path: str, base_dir: str) -> bytes:
    p = path if os.path.isabs(path) else os.path.join(base_dir, path)
    with open(p, "rb") as f:
        return f.read()


def _named(items, name: str, what: str) -> dict:
    for it in items or []:
        if it.get("name") == name:
            return it.get(what) or {}
    raise ConfigError(f"{what} {name!r} not found in kubeconfig")


def parse_kubeconfig(doc: dict, *, context: str | None = None, base_dir: str = "", name: str = "") -> ClusterConfig:
    ctx_name = context or doc.get("current-context")
    if not ctx_name:
        ctxs = doc.get("contexts") or []
        if len(ctxs) != 1:
            raise ConfigError("kubeconfig has no current-context")
        ctx_name = ctxs[0]["name"]
    ctx = _named(doc.get("contexts"), ctx_name, "context")
    cluster = _named(doc.get("clusters"), ctx.get("cluster", ""), "cluster")
    user = _named(doc.get("users"), ctx["user"], "user") if ctx.get("user") else {}
    server = cluster.get("server")
    if not server:
        raise ConfigError(f"cluster {ctx.get('cluster')!r} has no server")
    cfg = ClusterConfig(server=server.rstrip("/"), name=name or ctx_name, namespace=ctx.get("namespace"),
                        base_dir=base_dir)
    if cluster.get("certificate-authority-data"):
        cfg.ca_data = base64.b64decode(cluster["certificate-authority-data"])
    elif cluster.get("certificate-authority"):
        cfg.ca_data = _read(cluster["certificate-authority"], base_dir)
    cfg.insecure = bool(cluster.get("insecure-skip-tls-verify", False))
    cfg.tls_server_name = cluster.get("tls-server-name")
    cfg.proxy_url = cluster.get("proxy-url") or None
    if user.get("client-certificate-data"):
        cfg.client_cert_data = base64.b64decode(user["client-certificate-data"])
    elif user.get("client-certificate"):
        cfg.client_cert_data = _read(user["client-certificate"], base_dir)
    if user.get("client-key-data"):
        cfg.client_key_data = base64.b64decode(user["client-key-data"])
    elif user.get("client-key"):
        cfg.client_key_data = _read(user["client-key"], base_dir)
    cfg.token = user.get("token")
    if user.get("tokenFile"):
        tf = user["tokenFile"]
        cfg.token_file = tf if os.path.isabs(tf) else os.path.join(base_dir, tf)
    cfg.username, cfg.password = user.get("username"), user.get("password")
    ex = user.get("exec")
    if ex:
        cfg.exec = ExecConfig(command=ex["command"], args=list(ex.get("args") or []), env=list(ex.get("env") or []),
                              api_version=ex.get("apiVersion", "client.authentication.k8s.io/v1"),
                              provide_cluster_info=bool(ex.get("provideClusterInfo", False)),
                              interactive_mode=ex.get("interactiveMode", "Never"))
    return cfg


def load_kubeconfig(path: str, context: str | None = None, name: str = "") -> ClusterConfig:
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    return parse_kubeconfig(doc, context=context, base_dir=os.path.dirname(os.path.abspath(path)), name=name)


def in_cluster_config() -> ClusterConfig:
    host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
    if not host or not port:
        raise ConfigError("unable to load in-cluster configuration, KUBERNETES_SERVICE_HOST and "
                          "KUBERNETES_SERVICE_PORT must be defined")
    if ":" in host:
        host = f"[{host}]"
    cfg = ClusterConfig(server=f"https://{host}:{port}", name="in-cluster", token_file=os.path.join(SA_DIR, "token"))
    ca = os.path.join(SA_DIR, "ca.crt")
    if os.path.exists(ca):
        with open(ca, "rb") as f:
            cfg.ca_data = f.read()
    ns = os.path.join(SA_DIR, "namespace")
    if os.path.exists(ns):
        with open(ns) as f:
            cfg.namespace = f.read().strip()
    return cfg


def build_config(path: str | None) -> ClusterConfig:
    """clientcmd.BuildConfigFromFlags("", path): explicit file, else in-cluster, else $KUBECONFIG / ~/.kube/config."""
    if path:
        return load_kubeconfig(path)
    try:
        return in_cluster_config()
    except ConfigError:
        pass
    for cand in (os.environ.get("KUBECONFIG", "").split(os.pathsep)[0], os.path.expanduser("~/.kube/config")):
        if cand and os.path.exists(cand):
            return load_kubeconfig(cand)
    raise ConfigError("no kubeconfig path given, not running in-cluster, and no default kubeconfig found")


def render_kubeconfig(server: str, name: str, *, token: str | None = None, ca_data: bytes | None = None,
                      insecure: bool = False, namespace: str | None = None, exec_cfg: dict | None = None,
                      client_cert_data: bytes | None = None, client_key_data: bytes | None = None,
                      tls_server_name: str | None = None, proxy_url: str | None = None) -> str:
    """Write a minimal single-context kubeconfig (used by tests, benches and the Helm README example)."""
    cluster = {"server": server}
    if ca_data:
        cluster["certificate-authority-data"] = base64.b64encode(ca_data).decode()
    if insecure:
        cluster["insecure-skip-tls-verify"] = True
    if tls_server_name:
        cluster["tls-server-name"] = tls_server_name
    if proxy_url:
        cluster["proxy-url"] = proxy_url
    user: dict = {}
    if client_cert_data and client_key_data:  # x509 client auth, as in a kind cluster's admin kubeconfig
        user["client-certificate-data"] = base64.b64encode(client_cert_data).decode()
        user["client-key-data"] = base64.b64encode(client_key_data).decode()
    if token:
        user["token"] = token
    if exec_cfg:
        user["exec"] = exec_cfg
    ctx = {"cluster": name, "user": name}
    if namespace:
        ctx["namespace"] = namespace
    doc = {"apiVersion": "v1", "kind": "Config", "current-context": name,
           "clusters": [{"name": name, "cluster": cluster}], "users": [{"name": name, "user": user}],
           "contexts": [{"name": name, "context": ctx}]}
    return yaml.safe_dump(doc, sort_keys=False)


class CredentialSource:
    """Resolves the bearer token / client cert for a config, running exec plugins when needed."""

    def __init__(self, cfg: ClusterConfig):
        self.cfg = cfg
        self._token: str | None = None
        self._cert: tuple | None = None
        self._expiry: float | None = None
        self._lock = asyncio.Lock()
        self.exec_runs = 0
        self._file_token: str | None = None
        self._file_read_at = -1e18

    # client-go re-reads a token file at most once a minute (transport.NewCachedFileTokenSource)
    FILE_TOKEN_PERIOD = 60.0

    def cached_token(self) -> tuple[bool, str | None]:
        """Synchronous fast path for the per-request Authorization header: (True, token) when no I/O or
        exec run is needed (static token, a token file read within the last minute, an unexpired exec
        credential), else (False, None) and the caller awaits `token()`."""
        cfg = self.cfg
        if cfg.exec is not None:
            if (self._token is not None or self._cert is not None) and not self._expired():
                return True, self._token
            return False, None
        if cfg.token:
            return True, cfg.token
        if cfg.token_file:
            if time.monotonic() - self._file_read_at < self.FILE_TOKEN_PERIOD:
                return True, self._file_token
            return False, None
        return True, None

    def _expired(self) -> bool:
        if self._expiry is None:
            return False
        return _dt.datetime.now(_dt.timezone.utc).timestamp() > self._expiry - 10

    async def token(self, force_refresh: bool = False) -> str | None:
        cfg = self.cfg
        if cfg.exec is not None:
            async with self._lock:
                if force_refresh or (self._token is None and self._cert is None) or self._expired():
                    await self._run_exec()
            return self._token
        if cfg.token:
            return cfg.token
        if cfg.token_file:
            if force_refresh or time.monotonic() - self._file_read_at >= self.FILE_TOKEN_PERIOD:
                try:
                    with open(cfg.token_file) as f:  # re-read periodically: projected SA tokens rotate
                        self._file_token = f.read().strip()
                except OSError:
                    self._file_token = None
                self._file_read_at = time.monotonic()
            return self._file_token
        return None

    async def exec_client_cert(self) -> tuple | None:
        if self.cfg.exec is None:
            return None
        await self.token()
        return self._cert

    async def _run_exec(self) -> None:
        ex = self.cfg.exec
        env = dict(os.environ)
        for e in ex.env:
            env[e["name"]] = e.get("value", "")
        info = {"apiVersion": ex.api_version, "kind": "ExecCredential",
                "spec": {"interactive": False}}
        if ex.provide_cluster_info:
            info["spec"]["cluster"] = {"server": self.cfg.server, "insecure-skip-tls-verify": self.cfg.insecure}
            if self.cfg.ca_data:
                info["spec"]["cluster"]["certificate-authority-data"] = base64.b64encode(self.cfg.ca_data).decode()
        env["KUBERNETES_EXEC_INFO"] = json.dumps(info)
        proc = await asyncio.create_subprocess_exec(ex.command, *ex.args, env=env, stdout=asyncio.subprocess.PIPE,
                                                    stderr=asyncio.subprocess.PIPE, stdin=asyncio.subprocess.DEVNULL)
        out, err = await proc.communicate()
        self.exec_runs += 1
        if proc.returncode != 0:
            raise ConfigError(f"exec plugin {ex.command} failed ({proc.returncode}): {err.decode(errors='replace')}")
        cred = json.loads(out)
        st = cred.get("status") or {}
        self._token = st.get("token")
        if st.get("clientCertificateData") and st.get("clientKeyData"):
            self._cert = (st["clientCertificateData"].encode(), st["clientKeyData"].encode())
        exp = st.get("expirationTimestamp")
        if exp:
            self._expiry = _dt.datetime.fromisoformat(exp.replace("Z", "+00:00")).timestamp()
        else:
            self._expiry = None
