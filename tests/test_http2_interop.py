"""HTTP/2 interop with independent implementations ("next 2").

Until round 5 every HTTP/2 peer in the suite was this repository's own (the C++ and Python clients, the fake
apiserver's server, one HPACK header for both sides).  Here each side meets another implementation:

* Node's `http2` module (nghttp2) as a reverse proxy in front of the fake apiserver (tests/interop/h2proxy.js):
  MAX_CONCURRENT_STREAMS 50 and a 64 KiB initial window, over h2c prior knowledge and over TLS with ALPN.  The
  C++ executor's client (`build/tools/ncc-h2probe`, compiled from native/executor/http.hpp) and the Python pool
  (`ncc/kube/h2client.py`) run lists, watches, creates and updates through it, with bodies above 64 KiB and more
  streams than the proxy allows at once; the proxy then sends GOAWAY mid-run and both clients carry on on a new
  connection.  The whole C++ executor (`ncc/bin/ncc-executor`) syncs templates through it.
* grpcio's server (gRPC core, chttp2) as a second peer for the Python pool: 200 concurrent POSTs against 16
  streams, a 300 KB body through 64 KiB windows, and `server.stop(grace)` (GOAWAY) under load.
* curl (libcurl + nghttp2) against the fake apiserver's own HTTP/2 server: h2c prior knowledge, TLS + ALPN with
  client certificates, the HTTP/1.1 fallback, multiplexed parallel transfers and a 300 KB POST/GET.

Each group skips when its tool is absent.  A strict peer catches what self-tests cannot: nghttp2 resets a stream
whose pseudo-header fields follow a regular field (RFC 9113 §8.3), the production-fatal mismatch found by
reasoning in round 5 (commit a69d9eb).  Reference transport: client-go's, /root/reference/main.go:52-68.
"""
import asyncio
import base64
import json
import os
import shutil
import subprocess
import sys

import pytest

from ncc.api import resources as R
from ncc.fakeapi.server import FakeApiServer
from ncc.kube.kubeconfig import ClusterConfig
from ncc.kube.rest import RestClient
from ncc.testing.workload import make_secret

NS = "nexus"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROXY_JS = os.path.join(ROOT, "tests", "interop", "h2proxy.js")
NODE = shutil.which("node") or shutil.which("nodejs")
CURL = shutil.which("curl")


def _node_has_http2() -> bool:
    if NODE is None:
        return False
    r = subprocess.run([NODE, "-e", "require('http2')"], capture_output=True, timeout=30)
    return r.returncode == 0


needs_node = pytest.mark.skipif(not _node_has_http2(), reason="node with the http2 module is not installed")


def _pki(tmp_path):
    from ncc.testing.pki import PKIUnavailable, make_pki
    try:
        return make_pki(str(tmp_path / "pki"))
    except PKIUnavailable as e:
        pytest.skip(str(e))


def _probe():
    sys.path.insert(0, os.path.join(ROOT, "native"))
    import build
    try:
        return build.build_tools()
    except Exception as e:  # noqa: BLE001
        pytest.skip(f"ncc-h2probe not buildable here: {e}")


class NodeProxy:
    def __init__(self, upstream: str, mode: str, pki=None):
        self.upstream, self.mode, self.pki = upstream, mode, pki
        self.proc = None

    async def start(self) -> str:
        args = [NODE, PROXY_JS, self.upstream, self.mode]
        if self.mode == "tls":
            args += [self.pki.server_cert, self.pki.server_key]
        self.proc = await asyncio.create_subprocess_exec(*args, stdin=asyncio.subprocess.PIPE,
                                                         stdout=asyncio.subprocess.PIPE)
        port = json.loads(await asyncio.wait_for(self.proc.stdout.readline(), 30))["port"]
        return f"{'https' if self.mode == 'tls' else 'http'}://127.0.0.1:{port}"

    async def command(self, what: str) -> dict:
        self.proc.stdin.write(what.encode() + b"\n")
        await self.proc.stdin.drain()
        return json.loads(await asyncio.wait_for(self.proc.stdout.readline(), 10))

    async def stop(self):
        if self.proc is not None and self.proc.returncode is None:
            self.proc.stdin.close()
            try:
                await asyncio.wait_for(self.proc.wait(), 5)
            except asyncio.TimeoutError:
                self.proc.kill()
                await self.proc.wait()


async def _upstream():
    srv = FakeApiServer(http2=False)  # the proxy speaks HTTP/1.1 to it: every HTTP/2 byte is nghttp2's
    return srv, await srv.start()


def _secret_body(name: str, size: int = 0) -> str:
    obj = make_secret(name, NS)
    if size:
        obj["data"] = {"blob": base64.b64encode(os.urandom(size * 3 // 4)).decode()}
    return json.dumps(obj, separators=(",", ":"))


# ------------------------------------------------------------------------------------- C++ client via nghttp2
@needs_node
@pytest.mark.parametrize("mode", ["h2c", "tls"])
async def test_cpp_client_through_nghttp2_proxy(tmp_path, mode):
    probe = _probe()
    pki = _pki(tmp_path) if mode == "tls" else None
    srv, up = await _upstream()
    proxy = NodeProxy(up, mode, pki)
    url = await proxy.start()
    try:
        base = f"/api/v1/namespaces/{NS}/secrets"
        steps = [f"POST {base} {_secret_body(f's{i}')}" for i in range(80)]  # 80 streams against 50 allowed
        steps += ["WAIT", f"POST {base} {_secret_body('big', 160 * 1024)}", "WAIT"]  # a body past the 64 KiB window
        steps += [f"GET {base}/s{i}" for i in range(0, 80, 7)]
        steps += [f"WATCH {base}?watch=1&resourceVersion=0&timeoutSeconds=1", f"GET {base}", "WAIT"]
        steps += [f"PUT {base}/big {_secret_body('big', 100 * 1024)}", "WAIT"]
        args = [probe, url, "1" if mode == "tls" else "2", "--pool", "4"] + (["--ca", pki.ca_cert] if pki else [])
        p = await asyncio.create_subprocess_exec(*args, stdin=asyncio.subprocess.PIPE, stdout=asyncio.subprocess.PIPE,
                                                 stderr=asyncio.subprocess.PIPE)
        out, err = await asyncio.wait_for(p.communicate("\n".join(steps).encode() + b"\n"), 60)
        lines = [json.loads(x) for x in out.decode().splitlines()]
        stats, res = lines[-1]["stats"], {r["i"]: r for r in lines[:-1]}
        assert stats["http2"] == 1 and stats["h2_streams"] >= 95, stats
        assert all(res[i].get("status") == 201 for i in range(80)), [res[i] for i in range(80) if "error" in res[i]]
        assert res[80]["status"] == 201  # the 160 KB create, through 64 KiB stream windows
        gets = [res[i] for i in range(81, 81 + len(range(0, 80, 7)))]
        assert all(g["status"] == 200 for g in gets)
        watch, listing, put = res[81 + len(gets)], res[82 + len(gets)], res[83 + len(gets)]
        assert watch.get("lines", 0) >= 81, watch  # every ADDED event of the initial state, then the stream ended
        assert listing["status"] == 200 and listing["bytes"] > 160 * 1024
        assert put["status"] == 200
        assert srv.state.count(R.SECRETS) == 81
    finally:
        await proxy.stop()
        await srv.stop()


@needs_node
async def test_cpp_client_carries_on_after_goaway(tmp_path):
    probe = _probe()
    srv, up = await _upstream()
    proxy = NodeProxy(up, "h2c")
    url = await proxy.start()
    try:
        base = f"/api/v1/namespaces/{NS}/secrets"
        steps = [f"POST {base} {_secret_body(f'a{i}')}" for i in range(20)] + ["WAIT", "SLEEP 1500"]
        steps += [f"POST {base} {_secret_body(f'b{i}')}" for i in range(20)] + ["WAIT"]
        p = await asyncio.create_subprocess_exec(probe, url, "2", stdin=asyncio.subprocess.PIPE,
                                                 stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE)
        p.stdin.write("\n".join(steps).encode() + b"\n")
        p.stdin.close()
        for _ in range(200):  # the first 20 are in: GOAWAY while the client sleeps on its open connection
            if srv.state.count(R.SECRETS) >= 20:
                break
            await asyncio.sleep(0.02)
        assert (await proxy.command("goaway"))["goaway"] == 1
        out = await asyncio.wait_for(p.stdout.read(), 60)
        await p.wait()
        lines = [json.loads(x) for x in out.decode().splitlines()]
        stats = lines[-1]["stats"]
        assert [r.get("status") for r in lines[:-1]] == [201] * 40, lines
        assert stats["h2_goaways"] == 1 and stats["h2_goaway_errors"] == 0 and stats["http2"] == 1
        assert srv.state.count(R.SECRETS) == 40
    finally:
        await proxy.stop()
        await srv.stop()


# ----------------------------------------------------------------------------------- Python pool via nghttp2
@needs_node
@pytest.mark.parametrize("mode", ["h2c", "tls"])
async def test_python_pool_through_nghttp2_proxy(tmp_path, mode):
    pki = _pki(tmp_path) if mode == "tls" else None
    srv, up = await _upstream()
    proxy = NodeProxy(up, mode, pki)
    url = await proxy.start()
    cfg = ClusterConfig(server=url, ca_data=pki.ca_data if pki else None)
    c = RestClient(cfg, http2="auto" if mode == "tls" else "on")
    try:
        seen = []

        async def watch():
            async for lines in c.watch_raw_batches(R.SECRETS, NS, resource_version="0"):
                seen.extend(lines)
        w = asyncio.ensure_future(watch())
        await asyncio.gather(*[c.create(R.SECRETS, NS, make_secret(f"s{i}", NS)) for i in range(120)])
        big = make_secret("big", NS)
        big["data"] = {"blob": base64.b64encode(os.urandom(300 * 1024)).decode()}
        await c.create(R.SECRETS, NS, big)  # 400 KB of JSON through 64 KiB windows
        got = await c.get(R.SECRETS, NS, "big")
        assert got["data"] == big["data"]
        got["data"] = {"k": "dmFsdWU="}
        assert (await c.update(R.SECRETS, NS, got))["data"] == {"k": "dmFsdWU="}
        assert len((await c.list(R.SECRETS, NS))["items"]) == 121
        assert c.protocol == "h2"
        for _ in range(200):
            if len(seen) >= 122:
                break
            await asyncio.sleep(0.02)
        assert len(seen) >= 122  # 121 ADDED + the update, streamed through the proxy
        # GOAWAY: the pool moves to a new connection; the watch's stream on the old one ends and is not lost
        before = c._pool.opened
        assert (await proxy.command("goaway"))["goaway"] >= 1
        await asyncio.sleep(0.1)
        await asyncio.gather(*[c.create(R.SECRETS, NS, make_secret(f"t{i}", NS)) for i in range(30)])
        assert c._pool.opened > before and c._pool.stats["h2_goaways"] >= 1
        assert srv.state.count(R.SECRETS) == 151
        w.cancel()
        await asyncio.gather(w, return_exceptions=True)
    finally:
        await c.close()
        await proxy.stop()
        await srv.stop()


# ------------------------------------------------------------------------ the whole C++ executor via nghttp2
@needs_node
async def test_native_executor_syncs_through_nghttp2_proxy(tmp_path, monkeypatch):
    """The C++ executor writing to a shard whose only HTTP/2 speaker is nghttp2: 40 templates with 160 KB
    Secrets land, a GOAWAY mid-run changes nothing, and an update wave after it propagates."""
    from ncc.app import App
    from ncc.controller.native_executor import binary_path
    from ncc.kube.kubeconfig import render_kubeconfig
    from ncc.testing.env import FakeEnvironment
    from ncc.testing.workload import make_template
    if binary_path() is None:
        pytest.skip("the C++ executor is not built")
    monkeypatch.delenv("NCC_EXECUTOR_IMPL", raising=False)
    env = await FakeEnvironment(1, str(tmp_path), http2=False).start()
    cc, sc = env.controller_client(), env.shard_client(0)  # (the test reads the shard directly, over HTTP/1.1)
    proxy = NodeProxy(env.shard_urls[0], "h2c")
    url = await proxy.start()
    with open(os.path.join(env.shard_dir, "shard-0.kubeconfig"), "w") as f:
        f.write(render_kubeconfig(url, "shard-0"))  # the controller's view of the shard: nghttp2
    app = App(env.app_config(mode="native", executor_impl="native", client_http2="on", failure_rate_max_delay=0.2,
                             health_bind_address="127.0.0.1:0"))
    stop = asyncio.Event()
    try:
        T = 40
        for i in range(T):
            s = make_secret(f"s{i}", NS)
            s["data"] = {"blob": base64.b64encode(os.urandom(120 * 1024)).decode()}
            await cc.create(R.SECRETS, NS, s)
            await cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=[f"s{i}"], configmaps=[]))
        await app.build()
        task = asyncio.ensure_future(app.run(stop))
        await asyncio.wait_for(app.controller.ready.wait(), 20)
        assert app.executor_impl == "native"

        async def landed(n, pred=lambda o: True):
            for _ in range(400):
                items = (await sc.list(R.SECRETS, NS))["items"]
                if sum(1 for o in items if pred(o)) >= n:
                    return True
                await asyncio.sleep(0.05)
            return False
        assert await landed(T) and len((await sc.list(R.TEMPLATES, NS))["items"]) == T
        assert (await proxy.command("goaway"))["goaway"] >= 1
        for i in range(T):
            s = await cc.get(R.SECRETS, NS, f"s{i}")
            s["data"] = {"v": base64.b64encode(b"wave-2").decode()}
            await cc.update(R.SECRETS, NS, s)
        assert await landed(T, lambda o: (o.get("data") or {}).get("v") == base64.b64encode(b"wave-2").decode())
        flow = {}
        for _ in range(100):  # the executor's next status message carries its client counters
            st = app.debug_state().get("executors") or {}
            flow = next(iter(((v.get("status") or {}).get("flow") or {}).get("shard-0", {}) for v in st.values()), {})
            if flow.get("h2_goaways", 0) >= 1:
                break
            await asyncio.sleep(0.1)
        assert flow.get("http2") == 1 and flow.get("h2_goaways", 0) >= 1, flow
        stats = await proxy.command("stats")
        assert stats["streams"] >= 2 * T  # the writes went through nghttp2 as HTTP/2 streams
    finally:
        stop.set()
        if "task" in locals():
            await asyncio.wait_for(task, 20)
        await proxy.stop()
        await env.stop()


# ------------------------------------------------------------------------------------- grpcio (chttp2) peer
def _grpc_frame(payload: bytes) -> bytes:
    return b"\x00" + len(payload).to_bytes(4, "big") + payload


async def test_python_pool_against_grpc_server():
    grpc = pytest.importorskip("grpc")
    from concurrent import futures

    from ncc.kube import h2client

    def echo(request, context):
        return request

    server = grpc.server(futures.ThreadPoolExecutor(max_workers=8),
                         options=[("grpc.max_concurrent_streams", 16), ("grpc.http2.bdp_probe", 0),
                                  ("grpc.max_receive_message_length", 8 << 20),
                                  ("grpc.max_send_message_length", 8 << 20)])
    handler = grpc.method_handlers_generic_handler("ncc.Test", {"Echo": grpc.unary_unary_rpc_method_handler(echo)})
    server.add_generic_rpc_handlers((handler,))
    port = server.add_insecure_port("127.0.0.1:0")
    server.start()
    pool = h2client.H2Pool(f"http://127.0.0.1:{port}", prior_knowledge=True, max_size=2, connect_timeout=5)
    hdr = {"content-type": "application/grpc", "te": "trailers"}
    try:
        async def call(payload: bytes):
            r = await pool.request("POST", "/ncc.Test/Echo", hdr, _grpc_frame(payload), timeout=20)
            assert r.status == 200
            return r.body[5:]
        outs = await asyncio.gather(*[call(b"x%d" % i) for i in range(200)])  # 200 streams against 16 at a time
        assert outs == [b"x%d" % i for i in range(200)]
        big = os.urandom(300 * 1024)
        assert await call(big) == big  # through gRPC core's 64 KiB windows, both ways
        assert pool.conns and all(c.peer_max_streams == 16 for c in pool.conns)
        # graceful stop under load: GOAWAY; the streams it lets finish finish
        pending = [asyncio.ensure_future(call(b"late%d" % i)) for i in range(16)]
        await asyncio.sleep(0.05)
        stopped = server.stop(grace=3)
        res = await asyncio.gather(*pending, return_exceptions=True)
        ok = [r for r in res if not isinstance(r, BaseException)]
        assert ok, res
        await asyncio.get_running_loop().run_in_executor(None, stopped.wait)
    finally:
        pool.close()
        server.stop(None)


# ----------------------------------------------------------------------------- curl against the fake apiserver
needs_curl = pytest.mark.skipif(CURL is None or "HTTP2" not in subprocess.run(
    [CURL or "true", "--version"], capture_output=True, text=True).stdout, reason="curl with HTTP/2 not installed")


def _curl(*args, data: bytes | None = None) -> subprocess.CompletedProcess:
    return subprocess.run([CURL, "-sS", *args], input=data, capture_output=True, timeout=60)


@needs_curl
async def test_curl_against_fake_apiserver(tmp_path):
    from ncc.testing.pki import PKIUnavailable, make_pki
    srv = FakeApiServer(http2=True)
    url = await srv.start()
    base = f"{url}/api/v1/namespaces/{NS}/secrets"
    loop = asyncio.get_running_loop()

    async def curl(*args, data=None):
        return await loop.run_in_executor(None, lambda: _curl(*args, data=data))
    try:
        r = await curl("--http2-prior-knowledge", "-w", "\n%{http_version}", base)
        body, ver = r.stdout.rsplit(b"\n", 1)
        assert r.returncode == 0 and ver == b"2" and json.loads(body)["kind"] == "SecretList"
        big = _secret_body("big", 300 * 1024).encode()
        r = await curl("--http2-prior-knowledge", "-X", "POST", "-H", "Content-Type: application/json",
                       "--data-binary", "@-", "-w", "\n%{http_code}", base, data=big)
        assert r.stdout.rsplit(b"\n", 1)[1] == b"201", r.stdout[-300:]
        r = await curl("--http2-prior-knowledge", f"{base}/big")
        assert json.loads(r.stdout)["data"] == json.loads(big)["data"]
        # many transfers multiplexed on one connection
        urls = sum((["-o", "/dev/null", f"{base}/big"] for _ in range(12)), [])
        r = await curl("--http2-prior-knowledge", "--parallel", "--parallel-max", "12",
                       "-w", "%{http_code} %{num_connects}\n", *urls)
        codes = r.stdout.decode().split()
        assert codes[0::2] == ["200"] * 12 and sum(int(n) for n in codes[1::2]) == 1, codes
        r = await curl("--http1.1", "-w", "\n%{http_version}", base)
        assert r.stdout.rsplit(b"\n", 1)[1] == b"1.1"
    finally:
        await srv.stop()
    # TLS: ALPN negotiates h2; the server requires a client certificate (kube-apiserver --client-ca-file)
    try:
        pki = make_pki(str(tmp_path / "pki"))
    except PKIUnavailable as e:
        pytest.skip(str(e))
    srv = FakeApiServer(http2=True)
    url = await srv.start(ssl_context=pki.server_context())
    try:
        tls = ["--cacert", pki.ca_cert, "--cert", pki.client_cert, "--key", pki.client_key]
        r = await curl(*tls, "--http2", "-w", "\n%{http_version}", f"{url}/api/v1/namespaces/{NS}/configmaps")
        assert r.returncode == 0 and r.stdout.rsplit(b"\n", 1)[1] == b"2", r.stderr
        r = await curl(*tls, "--http1.1", "-w", "\n%{http_version}", f"{url}/api/v1/namespaces/{NS}/configmaps")
        assert r.stdout.rsplit(b"\n", 1)[1] == b"1.1"
        r = await curl("--cacert", pki.ca_cert, "--http2", f"{url}/api/v1/namespaces/{NS}/configmaps")
        assert r.returncode != 0  # no client certificate: refused in the handshake
    finally:
        await srv.stop()
