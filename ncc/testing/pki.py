"""Throwaway PKI for TLS tests and local clusters: a CA, a server certificate and a client certificate.

kind clusters (the reference CI's substrate, .github/workflows/build.yaml:44-66) serve HTTPS with a
cluster CA and hand out kubeconfigs with `certificate-authority-data` plus an x509 client
certificate (`client-certificate-data`/`client-key-data`).  This module reproduces that shape with
the `openssl` CLI so the transport, kubeconfig and fake apiserver can be tested end to end over
mutual TLS.  Nothing here is used on a production path.
"""
from __future__ import annotations

import os
import shutil
import ssl
import subprocess
from dataclasses import dataclass


class PKIUnavailable(RuntimeError):
    pass


@dataclass
class PKI:
    dir: str
    ca_cert: str
    server_cert: str
    server_key: str
    client_cert: str
    client_key: str

    def read(self, path: str) -> bytes:
        with open(path, "rb") as f:
            return f.read()

    @property
    def ca_data(self) -> bytes:
        return self.read(self.ca_cert)

    @property
    def client_cert_data(self) -> bytes:
        return self.read(self.client_cert)

    @property
    def client_key_data(self) -> bytes:
        return self.read(self.client_key)

    def server_context(self, require_client_cert: bool = True) -> ssl.SSLContext:
        """Server side: present the server certificate; with `require_client_cert`, reject clients that do
        not present a certificate signed by the CA (kube-apiserver `--client-ca-file`)."""
        ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
        ctx.load_cert_chain(self.server_cert, self.server_key)
        if require_client_cert:
            ctx.load_verify_locations(cafile=self.ca_cert)
            ctx.verify_mode = ssl.CERT_REQUIRED
        return ctx


def _openssl(*args: str, cwd: str) -> None:
    r = subprocess.run(["openssl", *args], cwd=cwd, capture_output=True, text=True, timeout=60)
    if r.returncode != 0:
        raise PKIUnavailable(f"openssl {' '.join(args[:2])} failed: {r.stderr.strip()[-500:]}")


def make_pki(directory: str, *, server_names: tuple = ("localhost", "kube.test"),
             server_ips: tuple = ("127.0.0.1",), client_cn: str = "nexus-configuration-controller",
             client_org: str = "system:masters") -> PKI:
    """Generate CA + server + client key pairs (EC P-256, 1 day) under `directory`."""
    if shutil.which("openssl") is None:
        raise PKIUnavailable("openssl not found")
    os.makedirs(directory, exist_ok=True)
    d = directory
    _openssl("ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", "ca.key", cwd=d)
    _openssl("req", "-x509", "-new", "-key", "ca.key", "-sha256", "-days", "1", "-subj", "/CN=ncc-test-ca",
             "-addext", "basicConstraints=critical,CA:TRUE", "-addext", "keyUsage=critical,keyCertSign,cRLSign",
             "-out", "ca.crt", cwd=d)
    san = ",".join([f"DNS:{n}" for n in server_names] + [f"IP:{ip}" for ip in server_ips])
    leaves = (("server", "/CN=kube-apiserver", f"subjectAltName={san}\nextendedKeyUsage=serverAuth\n"),
              ("client", f"/O={client_org}/CN={client_cn}", "extendedKeyUsage=clientAuth\n"))
    for name, subj, ext in leaves:
        _openssl("ecparam", "-name", "prime256v1", "-genkey", "-noout", "-out", f"{name}.key", cwd=d)
        _openssl("req", "-new", "-key", f"{name}.key", "-subj", subj, "-out", f"{name}.csr", cwd=d)
        with open(os.path.join(d, f"{name}.ext"), "w") as f:
            f.write(ext)
        _openssl("x509", "-req", "-in", f"{name}.csr", "-CA", "ca.crt", "-CAkey", "ca.key", "-CAcreateserial",
                 "-days", "1", "-sha256", "-extfile", f"{name}.ext", "-out", f"{name}.crt", cwd=d)
    for p in os.listdir(d):
        if p.endswith(".key"):
            os.chmod(os.path.join(d, p), 0o600)
    j = lambda p: os.path.join(d, p)  # noqa: E731
    return PKI(d, j("ca.crt"), j("server.crt"), j("server.key"), j("client.crt"), j("client.key"))
