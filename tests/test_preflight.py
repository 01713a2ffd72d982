"""`python -m ncc --check-shards` (ncc/preflight.py): the deployment preflight of docs/MIGRATION.md."""
import json
import os

from ncc.preflight import check
from ncc.testing.env import FakeEnvironment


async def test_preflight_reports_each_cluster_and_names_the_failure(tmp_path):
    env = await FakeEnvironment(3, str(tmp_path)).start()
    try:
        cfg = env.app_config(mode="native")
        ok = await check(cfg)
        assert [r["cluster"] for r in ok] == ["controller", "shard-0", "shard-1", "shard-2"]
        assert all(r["ok"] for r in ok), ok
        assert all(r["protocol"] == "http/1.1" for r in ok)  # cleartext with client-http2 auto
        h2 = {r["cluster"]: r for r in await check(env.app_config(mode="native", client_http2="on"))}
        # `on` adds prior knowledge for the shards; the controller cluster negotiates (ALPN on TLS only)
        assert all(r["ok"] for r in h2.values()) and h2["controller"]["protocol"] == "http/1.1", h2
        assert all(h2[f"shard-{i}"]["protocol"] == "h2" for i in range(3)), h2
        # shard-1's credentials may not list Secrets; shard-2 lacks the workgroup CRD; a broken kubeconfig
        env.shard_servers[1].faults.update({"rules": [{"method": "GET", "resource": "secrets", "code": 403,
                                                       "message": "secrets is forbidden"}]})
        env.shard_servers[2].faults.update({"rules": [{"method": "GET", "resource": "nexusalgorithmworkgroups",
                                                       "code": 404, "message": "the server could not find "
                                                                                 "the requested resource"}]})
        with open(os.path.join(env.shard_dir, "broken.kubeconfig"), "w") as f:
            f.write("not: [a kubeconfig")
        res = {r["cluster"]: r for r in await check(cfg)}
        assert res["shard-0"]["ok"] and res["controller"]["ok"]
        assert res["shard-1"]["kinds"]["secrets"].startswith("Forbidden (403)")
        assert res["shard-1"]["kinds"]["configmaps"] == "ok"
        assert res["shard-2"]["kinds"]["nexusalgorithmworkgroups"].startswith("NotFound (404)")
        assert not res["broken"]["ok"] and res["broken"]["error"]
    finally:
        await env.stop()


def test_check_shards_flag_exit_status(tmp_path, monkeypatch, capsys):
    """The flag runs the preflight instead of the controller and exits 1 when a cluster fails (here: no
    shard kubeconfigs at all)."""
    from ncc import app
    (tmp_path / "appconfig.yaml").write_text(f"shard-config-path: {tmp_path / 'none'}\n"
                                             f"controller-config-path: {tmp_path / 'missing.kubeconfig'}\n")
    assert app.main(["--config-dir", str(tmp_path), "-check-shards"]) == 1
    lines = [json.loads(x) for x in capsys.readouterr().out.strip().splitlines()]
    assert lines[-1]["summary"] == "failed" and lines[-1]["shards"] == 0


def test_malformed_appconfig_is_a_configuration_error(tmp_path, capsys):
    from ncc import app
    (tmp_path / "appconfig.yaml").write_text("alias: a: b\n")
    assert app.main(["--config-dir", str(tmp_path), "--version"]) == 0  # --version needs no config
    assert app.main(["--config-dir", str(tmp_path), "--check-shards"]) == 1
    assert "configuration error" in capsys.readouterr().err


async def test_unreachable_cluster_is_reported_once(tmp_path):
    import socket

    from ncc.preflight import check_cluster
    from ncc.kube.kubeconfig import ClusterConfig
    from ncc.kube.rest import RestClient
    with socket.socket() as s:  # a port nothing listens on
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    client = RestClient(ClusterConfig(server=f"http://127.0.0.1:{port}"), pool_size=1, cluster_name="dead")
    try:
        r = await check_cluster("dead", client, "nexus", timeout=2.0)
    finally:
        await client.close()
    assert not r["ok"]
    first, *rest = r["kinds"].values()
    assert first.startswith("TransportError") and all(v.startswith("skipped") for v in rest), r
