"""Mutual TLS end to end: HTTPS apiservers with a cluster CA and x509 client auth, as in the kind clusters
of the reference CI (.github/workflows/build.yaml:44-66).  The kubeconfigs carry
`certificate-authority-data` + `client-certificate-data`/`client-key-data` (X7 shard loader,
main.go:52 controller config), and both transports must sync through them, watches included."""
import os

import pytest

from ncc.api import resources as R
from ncc.kube import errors as E
from ncc.kube.kubeconfig import load_kubeconfig, parse_kubeconfig
from ncc.kube.rest import RestClient
from ncc.testing.env import FakeEnvironment
from ncc.testing.pki import PKIUnavailable, make_pki
from ncc.testing.workload import make_configmap, make_secret, make_template

from test_e2e import NS, Running, _get, mutate, wait_for

try:
    import shutil
    HAVE_OPENSSL = shutil.which("openssl") is not None
except Exception:  # noqa: BLE001
    HAVE_OPENSSL = False

pytestmark = pytest.mark.skipif(not HAVE_OPENSSL, reason="openssl CLI needed to mint test certificates")


@pytest.mark.parametrize("mode,transport,subprocesses", [("native", "fast", False), ("native", "aiohttp", False),
                                                         ("compat", "fast", False), ("native", "fast", True)])
async def test_sync_over_mutual_tls(tmp_path, mode, transport, subprocesses):
    env = await FakeEnvironment(2, str(tmp_path), tls=True, subprocesses=subprocesses).start()
    assert env.controller_url.startswith("https://")
    cc = env.controller_client()
    scs = [env.shard_client(i) for i in range(2)]
    try:
        await cc.create(R.SECRETS, NS, make_secret("s0", NS))
        await cc.create(R.CONFIGMAPS, NS, make_configmap("c0", NS))
        await cc.create(R.TEMPLATES, NS, make_template(0, NS, secrets=["s0"], configmaps=["c0"]))
        async with Running(env, mode, transport=transport):
            for sc in scs:
                await wait_for(lambda sc=sc: _get(sc, R.TEMPLATES, "algo-00000"), timeout=5)
                await wait_for(lambda sc=sc: _get(sc, R.SECRETS, "s0"), timeout=5)
                await wait_for(lambda sc=sc: _get(sc, R.CONFIGMAPS, "c0"), timeout=5)
            # an update travels over the TLS watch streams too
            await mutate(cc, R.TEMPLATES, "algo-00000",
                         lambda o: o["spec"]["container"].__setitem__("versionTag", "v9"))
            for sc in scs:
                async def updated(sc=sc):
                    return (await sc.get(R.TEMPLATES, NS, "algo-00000"))["spec"]["container"]["versionTag"] == "v9"
                await wait_for(updated, timeout=5)
    finally:
        await cc.close()
        for sc in scs:
            await sc.close()
        await env.stop()


@pytest.mark.parametrize("transport", ["fast", "aiohttp"])
async def test_tls_failures_surface_as_transport_errors(tmp_path, transport):
    env = await FakeEnvironment(0, str(tmp_path), tls=True).start()
    try:
        good = load_kubeconfig(env.controller_kubeconfig)

        # 1) the right CA and a client certificate: accepted
        c = RestClient(good, transport=transport)
        try:
            assert (await c.list(R.SECRETS, NS))["items"] == []
        finally:
            await c.close()

        # 2) no client certificate: the apiserver rejects the handshake
        anon = load_kubeconfig(env.controller_kubeconfig)
        anon.client_cert_data = anon.client_key_data = None
        c = RestClient(anon, transport=transport, max_retries=0)
        try:
            with pytest.raises(E.TransportError):
                await c.list(R.SECRETS, NS)
        finally:
            await c.close()

        # 3) a CA that did not sign the server certificate: the client refuses the server
        other = make_pki(os.path.join(str(tmp_path), "other-pki"))
        wrong = load_kubeconfig(env.controller_kubeconfig)
        wrong.ca_data = other.ca_data
        c = RestClient(wrong, transport=transport, max_retries=0)
        try:
            with pytest.raises(E.TransportError):
                await c.list(R.SECRETS, NS)
        finally:
            await c.close()

        # 4) insecure-skip-tls-verify accepts any server certificate (client cert still presented)
        skip = load_kubeconfig(env.controller_kubeconfig)
        skip.ca_data, skip.insecure = other.ca_data, True
        c = RestClient(skip, transport=transport)
        try:
            assert (await c.list(R.SECRETS, NS))["items"] == []
        finally:
            await c.close()
    finally:
        await env.stop()


@pytest.mark.parametrize("server_name,ok", [("kube.test", True), ("not-in-the-cert.example", False)])
async def test_tls_server_name_overrides_verification_name(tmp_path, server_name, ok):
    env = await FakeEnvironment(0, str(tmp_path), tls=True).start()
    try:
        cfg = parse_kubeconfig({
            "current-context": "c", "contexts": [{"name": "c", "context": {"cluster": "c", "user": "u"}}],
            "clusters": [{"name": "c", "cluster": {"server": env.controller_url, "tls-server-name": server_name,
                                                   "certificate-authority": env.pki.ca_cert}}],
            "users": [{"name": "u", "user": {"client-certificate": env.pki.client_cert,
                                             "client-key": env.pki.client_key}}]})
        assert cfg.tls_server_name == server_name and cfg.ca_data == env.pki.ca_data
        c = RestClient(cfg, max_retries=0)
        try:
            if ok:
                assert (await c.list(R.CONFIGMAPS, NS))["items"] == []
            else:
                with pytest.raises(E.TransportError):
                    await c.list(R.CONFIGMAPS, NS)
        finally:
            await c.close()
    finally:
        await env.stop()


def test_pki_unavailable_is_reported(tmp_path, monkeypatch):
    monkeypatch.setattr("shutil.which", lambda _name: None)
    with pytest.raises(PKIUnavailable):
        make_pki(str(tmp_path))


async def test_http11_fallback_offers_only_http11_over_tls(tmp_path):
    """after the pool moves to HTTP/1.1 (HTTP_1_1_REQUIRED), its TLS connections must not offer h2
    by ALPN — a server that picks h2 whenever it is offered (the fake apiserver does, as Go's) would get
    HTTP/1.1 bytes on an h2 connection.  The control: the same pool falling back on its own HTTP/2 context
    (ALPN h2 + http/1.1, the round-5 behaviour) fails."""
    env = await FakeEnvironment(0, str(tmp_path), tls=True).start()
    try:
        for control in (False, True):
            c = RestClient(load_kubeconfig(env.controller_kubeconfig), http2="auto", max_retries=0)
            try:
                assert (await c.list(R.SECRETS, NS))["items"] == []
                pool = c._pool
                assert pool.protocol == "h2"
                if control:
                    pool.fallback_ssl = None  # fall back on the HTTP/2 context
                pool._downgrade("test")
                if control:
                    with pytest.raises(E.TransportError):
                        await c.list(R.SECRETS, NS)
                else:
                    for _ in range(3):
                        assert (await c.list(R.SECRETS, NS))["items"] == []
                    assert pool.protocol == "http/1.1" and pool.stats["h2_downgraded"] == 1
            finally:
                await c.close()
    finally:
        await env.stop()
