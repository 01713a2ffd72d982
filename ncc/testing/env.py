"""Fake multi-cluster environments: one controller apiserver + N shard apiservers + kubeconfigs.

The stand-in for the reference CI's two kind clusters (.github/workflows/build.yaml:44-66) and
for the 1/2/4/8-shard benchmark topologies.  Servers run either in-process (tests) or as
separate `python -m ncc.fakeapi` processes (benchmarks, so apiserver CPU is not charged to the
controller process).
"""
from __future__ import annotations

import asyncio
import os
import subprocess
import sys
import time

from ..config import AppConfig
from ..fakeapi.server import FakeApiServer
from ..kube.kubeconfig import load_kubeconfig, render_kubeconfig
from ..kube.rest import RestClient


def spawn_fakeapi(name: str, port_file: str, *, token: str | None = None, extra: list | None = None,
                  bookmark_interval: float = 5.0, pki=None) -> subprocess.Popen:
    if os.path.exists(port_file):
        os.remove(port_file)
    cmd = [sys.executable, "-m", "ncc.fakeapi", "--name", name, "--port-file", port_file,
           "--bookmark-interval", str(bookmark_interval), "--parent-pid", str(os.getpid())]
    if token:
        cmd += ["--token", token]
    if pki is not None:
        cmd += ["--tls-cert", pki.server_cert, "--tls-key", pki.server_key, "--tls-client-ca", pki.ca_cert]
    cmd += extra or []
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env = dict(os.environ)
    env["PYTHONPATH"] = root + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, env=env)


def wait_port_file(path: str, proc: subprocess.Popen | None = None, timeout: float = 60.0) -> str:
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout:
        if os.path.exists(path):
            with open(path) as f:
                url = f.read().strip()
            if url:
                return url
        if proc is not None and proc.poll() is not None:
            err = proc.stderr.read().decode(errors="replace") if proc.stderr else ""
            raise RuntimeError(f"fake apiserver exited early ({proc.returncode}): {err[-2000:]}")
        time.sleep(0.02)
    raise TimeoutError(f"fake apiserver did not publish {path} within {timeout}s")


class FakeEnvironment:
    def __init__(self, n_shards: int, workdir: str, *, namespace: str = "nexus", token: str | None = None,
                 subprocesses: bool = False, shard_prefix: str = "shard", bookmark_interval: float = 5.0,
                 tls: bool = False, tls_server_name: str | None = None, crd_dir: str | None = "default",
                 http2: bool = True):
        """`tls=True` serves every apiserver over HTTPS with mutual TLS (a throwaway CA, x509 client auth,
        like a kind cluster); `tls_server_name` additionally puts `tls-server-name` in the kubeconfigs.
        `crd_dir` ("default": the repository's deploy/crds) makes the apiservers validate custom-resource
        writes against the shipped CRD schemas, as a real apiserver does; None disables it.  `http2=False`:
        apiservers that speak HTTP/1.1 only (no ALPN h2, no prior-knowledge HTTP/2)."""
        self.n_shards = n_shards
        self.http2 = http2
        self.workdir = workdir
        self.namespace = namespace
        self.token = token
        self.subprocesses = subprocesses
        self.shard_names = [f"{shard_prefix}-{i}" for i in range(n_shards)]
        self.bookmark_interval = bookmark_interval
        self.controller_server: FakeApiServer | None = None
        self.shard_servers: list[FakeApiServer] = []
        self.procs: list[subprocess.Popen] = []
        self.controller_url = ""
        self.shard_urls: list[str] = []
        self.shard_dir = os.path.join(workdir, "shards")
        self.controller_kubeconfig = os.path.join(workdir, "controller.kubeconfig")
        self.tls = tls
        self.tls_server_name = tls_server_name
        if crd_dir == "default":
            root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            crd_dir = os.path.join(root, "deploy", "crds")
            crd_dir = crd_dir if os.path.isdir(crd_dir) else None
        self.crd_dir = crd_dir
        self.pki = None

    async def start(self) -> "FakeEnvironment":
        os.makedirs(self.shard_dir, exist_ok=True)
        names = ["controller"] + self.shard_names
        if self.tls:
            from .pki import make_pki
            self.pki = make_pki(os.path.join(self.workdir, "pki"))
        if self.subprocesses:
            files = []
            for n in names:
                pf = os.path.join(self.workdir, f"{n}.url")
                extra = (["--crd-dir", self.crd_dir] if self.crd_dir else []) + ([] if self.http2 else ["--no-http2"])
                self.procs.append(spawn_fakeapi(n, pf, token=self.token, bookmark_interval=self.bookmark_interval,
                                                pki=self.pki, extra=extra or None))
                files.append(pf)
            urls = [await asyncio.get_running_loop().run_in_executor(None, wait_port_file, f, p)
                    for f, p in zip(files, self.procs)]
        else:
            urls = []
            for n in names:
                s = FakeApiServer(name=n, token=self.token, bookmark_interval=self.bookmark_interval,
                                  crd_dir=self.crd_dir, http2=self.http2)
                s.record_writes = True
                urls.append(await s.start(ssl_context=self.pki.server_context() if self.pki else None))
                if n == "controller":
                    self.controller_server = s
                else:
                    self.shard_servers.append(s)
        self.controller_url, self.shard_urls = urls[0], urls[1:]
        with open(self.controller_kubeconfig, "w") as f:
            f.write(self.kubeconfig(self.controller_url, "controller"))
        for n, u in zip(self.shard_names, self.shard_urls):
            with open(os.path.join(self.shard_dir, f"{n}.kubeconfig"), "w") as f:
                f.write(self.kubeconfig(u, n))
        return self

    def kubeconfig(self, url: str, name: str, **kw) -> str:
        if self.pki is not None:
            kw.setdefault("ca_data", self.pki.ca_data)
            kw.setdefault("client_cert_data", self.pki.client_cert_data)
            kw.setdefault("client_key_data", self.pki.client_key_data)
            kw.setdefault("tls_server_name", self.tls_server_name)
        return render_kubeconfig(url, name, token=self.token, **kw)

    def app_config(self, mode: str = "native", **kw) -> AppConfig:
        cfg = AppConfig(alias="controller-cluster", controller_config_path=self.controller_kubeconfig,
                        shard_config_path=self.shard_dir, controller_namespace=self.namespace, mode=mode,
                        log_level="WARNING")
        for k, v in kw.items():
            setattr(cfg, k, v)
        return cfg

    def controller_client(self, **kw) -> RestClient:
        return RestClient(load_kubeconfig(self.controller_kubeconfig, name="controller"), **kw)

    def shard_client(self, i: int, **kw) -> RestClient:
        p = os.path.join(self.shard_dir, f"{self.shard_names[i]}.kubeconfig")
        return RestClient(load_kubeconfig(p, name=self.shard_names[i]), **kw)

    async def stop(self) -> None:
        for s in [self.controller_server] + self.shard_servers:
            if s is not None:
                await s.stop()
        for p in self.procs:
            if p.poll() is None:
                p.terminate()
        for p in self.procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        self.procs = []
