"""HTTP CONNECT proxies (ncc/kube/proxy.py), as client-go uses them: the kubeconfig's `proxy-url`, else
`HTTPS_PROXY` / `HTTP_PROXY` with `NO_PROXY` and loopback exempt; TLS and HTTP/2 run inside the tunnel.

* `proxy_for`'s rules, including Go's NO_PROXY forms (domains, leading dots, IPs, CIDRs, ports, `*`);
* the Python clients through a proxy to a TLS apiserver, over HTTP/2 (ALPN inside the tunnel) and HTTP/1.1,
  with proxy credentials, and a proxy that refuses;
* the C++ shard executor through a proxy (the coordinator renders the CONNECT request for it);
* the same over a SOCKS5 proxy (RFC 1928, username/password per RFC 1929), as Go's transport dials
  `socks5://` proxy URLs.
"""
import asyncio
import base64
import os

import pytest

from ncc.api import resources as R
from ncc.kube import errors as E
from ncc.kube.kubeconfig import load_kubeconfig
from ncc.kube.proxy import connect_request, proxy_for, socks5_connect_request
from ncc.kube.rest import RestClient
from ncc.testing.env import FakeEnvironment
from ncc.testing.workload import make_configmap, make_secret, make_template

NS = "nexus"


class ConnectProxy:
    """A minimal HTTP CONNECT proxy: checks Proxy-Authorization when `auth` is set, counts tunnels."""

    def __init__(self, auth: str | None = None):
        self.auth, self.tunnels, self.targets, self.server = auth, 0, [], None

    async def start(self) -> str:
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        return f"http://127.0.0.1:{self.server.sockets[0].getsockname()[1]}"

    async def _handle(self, r, w):
        try:
            head = await r.readuntil(b"\r\n\r\n")
        except (asyncio.IncompleteReadError, ConnectionError):
            w.close()
            return
        lines = head.decode("latin-1").split("\r\n")
        method, target, _ = lines[0].split(" ", 2)
        hdrs = {k.strip().lower(): v.strip() for k, _, v in (ln.partition(":") for ln in lines[1:] if ln)}
        if method != "CONNECT":
            w.write(b"HTTP/1.1 405 Method Not Allowed\r\n\r\n")
            w.close()
            return
        if self.auth is not None and hdrs.get("proxy-authorization") != "Basic " + base64.b64encode(
                self.auth.encode()).decode():
            w.write(b"HTTP/1.1 407 Proxy Authentication Required\r\n\r\n")
            await w.drain()
            w.close()
            return
        host, _, port = target.rpartition(":")
        ur, uw = await asyncio.open_connection(host.strip("[]"), int(port))
        self.tunnels += 1
        self.targets.append(target)
        w.write(b"HTTP/1.1 200 Connection established\r\n\r\n")
        await asyncio.gather(self._pump(r, uw), self._pump(ur, w))

    @staticmethod
    async def _pump(src, dst):
        try:
            while True:
                data = await src.read(65536)
                if not data:
                    break
                dst.write(data)
                await dst.drain()
        except (ConnectionError, asyncio.CancelledError):
            pass
        finally:
            dst.close()

    async def stop(self):
        self.server.close()


class Socks5Proxy:
    """A minimal SOCKS5 proxy (CONNECT only): username/password when `auth` ("user:pass") is set, else none."""

    def __init__(self, auth: str | None = None):
        self.auth, self.tunnels, self.targets, self.server = auth, 0, [], None

    async def start(self) -> str:
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        return f"socks5://127.0.0.1:{self.server.sockets[0].getsockname()[1]}"

    async def _handle(self, r, w):
        try:
            ver, n = await r.readexactly(2)
            methods = await r.readexactly(n)
            want = 2 if self.auth is not None else 0
            if ver != 5 or want not in methods:
                w.write(b"\x05\xff")
                w.close()
                return
            w.write(bytes([5, want]))
            if want == 2:
                _, ulen = await r.readexactly(2)
                user = await r.readexactly(ulen)
                pw = await r.readexactly((await r.readexactly(1))[0])
                ok = f"{user.decode()}:{pw.decode()}" == self.auth
                w.write(b"\x01" + (b"\x00" if ok else b"\x01"))
                if not ok:
                    w.close()
                    return
            _, cmd, _, atyp = await r.readexactly(4)
            if atyp == 3:
                host = (await r.readexactly((await r.readexactly(1))[0])).decode()
            else:
                import ipaddress
                host = str(ipaddress.ip_address(await r.readexactly(4 if atyp == 1 else 16)))
            port = int.from_bytes(await r.readexactly(2), "big")
        except (asyncio.IncompleteReadError, ConnectionError):
            w.close()
            return
        ur, uw = await asyncio.open_connection(host, port)
        self.tunnels += 1
        self.targets.append(f"{host}:{port}")
        w.write(b"\x05\x00\x00\x01\x7f\x00\x00\x01\x00\x00")
        await asyncio.gather(ConnectProxy._pump(r, uw), ConnectProxy._pump(ur, w))

    async def stop(self):
        self.server.close()


PROXIES = {"connect": ConnectProxy, "socks5": Socks5Proxy}


def test_proxy_for_follows_client_go():
    env = {"HTTPS_PROXY": "proxy.corp:3128", "HTTP_PROXY": "http://p80:8080",
           "NO_PROXY": "internal.corp,.svc,10.0.0.0/8,api.example:6443,[2001:db8::1]"}
    assert proxy_for("https://k8s.example:443", environ=env) == "http://proxy.corp:3128"  # scheme-less: http
    assert proxy_for("http://k8s.example", environ=env) == "http://p80:8080"
    assert proxy_for("https://a.internal.corp", environ=env) is None       # a domain and its subdomains
    assert proxy_for("https://internal.corp", environ=env) is None
    assert proxy_for("https://kubernetes.default.svc", environ=env) is None  # a leading dot: subdomains
    assert proxy_for("https://10.1.2.3:6443", environ=env) is None          # CIDR
    assert proxy_for("https://api.example:6443", environ=env) is None       # host and port
    assert proxy_for("https://api.example:443", environ=env) == "http://proxy.corp:3128"
    assert proxy_for("https://[2001:db8::1]:6443", environ=env) is None
    assert proxy_for("https://127.0.0.1:6443", environ=env) is None         # loopback is never proxied
    assert proxy_for("https://localhost:6443", environ=env) is None
    assert proxy_for("https://k8s.example", environ={"HTTPS_PROXY": "http://p", "NO_PROXY": "*"}) is None
    # "*.example.com" is Go's ".example.com": subdomains bypass, the domain itself does not
    star = {"HTTPS_PROXY": "http://p", "NO_PROXY": "*.shards.example"}
    assert proxy_for("https://eu-1.shards.example", environ=star) is None
    assert proxy_for("https://shards.example", environ=star) == "http://p"
    assert proxy_for("https://k8s.example", environ={}) is None
    # the kubeconfig's proxy-url wins, loopback included (client-go's rest.Config.Proxy)
    assert proxy_for("https://127.0.0.1:6443", "http://p:1", environ=env) == "http://p:1"
    req = connect_request("http://u%40x:p%3Aw@p:1", "k8s.example", 443).decode()
    assert req.startswith("CONNECT k8s.example:443 HTTP/1.1\r\nHost: k8s.example:443\r\n")
    assert "Proxy-Authorization: Basic " + base64.b64encode(b"u@x:p:w").decode() in req
    assert proxy_for("https://k8s.example", environ={"HTTPS_PROXY": "socks5://s:1080"}) == "socks5://s:1080"
    assert socks5_connect_request("10.0.0.1", 443) == b"\x05\x01\x00\x01\x0a\x00\x00\x01\x01\xbb"
    assert socks5_connect_request("[::1]", 6443)[3:4] == b"\x04"
    assert socks5_connect_request("k8s.example", 443) == b"\x05\x01\x00\x03\x0bk8s.example\x01\xbb"


@pytest.mark.parametrize("kind", sorted(PROXIES))
@pytest.mark.parametrize("http2", ["auto", "off"])
async def test_rest_client_through_a_proxy(tmp_path, http2, kind):
    env = await FakeEnvironment(0, str(tmp_path), tls=True).start()
    proxy = PROXIES[kind](auth="alice:s3cret")
    purl = await proxy.start()
    try:
        cfg = load_kubeconfig(env.controller_kubeconfig)
        cfg.proxy_url = purl.replace("://", "://alice:s3cret@")
        c = RestClient(cfg, http2=http2)
        try:
            await c.create(R.SECRETS, NS, make_secret("via-proxy", NS))
            assert (await c.get(R.SECRETS, NS, "via-proxy"))["metadata"]["name"] == "via-proxy"
            assert c.protocol == ("h2" if http2 == "auto" else "http/1.1")  # ALPN inside the tunnel
            assert proxy.tunnels >= 1 and all(t.endswith(env.controller_url.rsplit(":", 1)[1]) for t in proxy.targets)
        finally:
            await c.close()
        if kind == "socks5":  # aiohttp dials only http:// proxies: refused up front, not at the first request
            with pytest.raises(ValueError, match="socks5"):
                RestClient(cfg, transport="aiohttp")
            cfg.proxy_url = purl  # a proxy that wants credentials, offered none
            c = RestClient(cfg, http2=http2, max_retries=0)
            try:
                with pytest.raises(E.TransportError, match="authentication method"):
                    await c.list(R.SECRETS, NS)
            finally:
                await c.close()
        cfg.proxy_url = purl.replace("://", "://alice:wrong@")
        c = RestClient(cfg, http2=http2, max_retries=0)
        try:
            with pytest.raises(E.TransportError, match="refused CONNECT" if kind == "connect" else "rejected"):
                await c.list(R.SECRETS, NS)
        finally:
            await c.close()
    finally:
        await proxy.stop()
        await env.stop()


@pytest.mark.parametrize("kind", sorted(PROXIES) + ["socks5-open"])
@pytest.mark.parametrize("http2", ["auto", "off"])
async def test_shard_executor_through_a_proxy(tmp_path, monkeypatch, http2, kind):
    from ncc.app import App
    from ncc.controller.native_executor import binary_path
    if binary_path() is None:
        pytest.skip("ncc/bin/ncc-executor is not built")
    monkeypatch.setenv("NCC_STATUS_S", "0.2")
    env = await FakeEnvironment(1, str(tmp_path), tls=True).start()
    proxy = Socks5Proxy() if kind == "socks5-open" else PROXIES[kind](auth="exec:pw")
    purl = await proxy.start()
    cc = env.controller_client()
    stop, task = asyncio.Event(), None
    try:
        kc = os.path.join(env.shard_dir, "shard-0.kubeconfig")
        with open(kc) as f:
            text = f.read()
        with open(kc, "w") as f:  # the shard's kubeconfig names the proxy, with credentials
            f.write(text.replace("    server:", f"    proxy-url: {purl if proxy.auth is None else purl.replace('://', '://exec:pw@')}\n"
                                              "    server:", 1))
        assert load_kubeconfig(kc).proxy_url
        await cc.create(R.SECRETS, NS, make_secret("s0", NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap("c0", NS))
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=["s0"], configmaps=["c0"]))
        app = App(env.app_config(mode="native", executor_impl="native", failure_rate_max_delay=0.2,
                                 client_http2=http2))
        await app.build()
        task = asyncio.ensure_future(app.run(stop))
        for _ in range(600):
            if env.shard_servers[0].state.try_get(R.CONFIGMAPS, NS, "c0") is not None:
                break
            await asyncio.sleep(0.05)
        else:
            raise AssertionError("the executor never reached the shard through the proxy")
        # every shard connection of the executor (lists, watches, writes) went through the tunnel: over HTTP/2
        # (ALPN inside it) one or two, over HTTP/1.1 one per connection in use
        assert proxy.tunnels >= 1 and env.shard_servers[0]._http.conn_stats()["h2"]["connections"] == (
            0 if http2 == "off" else proxy.tunnels)
        assert env.shard_servers[0].state.try_get(R.TEMPLATES, NS, "algo-00000") is not None
    finally:
        stop.set()
        if task is not None:
            await task
        await cc.close()
        await proxy.stop()
        await env.stop()
