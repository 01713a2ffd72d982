"""Config loading (appconfig.yaml + env overlay + NEXUS__ env) and kubeconfig/exec-credential handling."""
import base64
import json
import os
import stat
import sys

import pytest

from ncc.api import resources as R
from ncc.config import AppConfig, config_to_env, load_config, parse_duration
from ncc.fakeapi.server import FakeApiServer
from ncc.kube import errors as E
from ncc.kube.kubeconfig import (ClusterConfig, ConfigError, CredentialSource, build_config, in_cluster_config,
                                 load_kubeconfig, parse_kubeconfig, render_kubeconfig)
from ncc.kube.rest import RestClient
from ncc.shards.loader import discover

REF_KEYS = ["alias", "controller-config-path", "shard-config-path", "controller-namespace", "log-level", "workers",
            "failure-rate-base-delay", "failure-rate-max-delay", "rate-limit-elements-per-second",
            "rate-limit-elements-burst"]


@pytest.mark.parametrize("text,sec", [("30ms", 0.03), ("5s", 5.0), ("1m30s", 90.0), ("1h", 3600.0), ("2", 2.0),
                                      ("1.5s", 1.5), ("-1s", -1.0), ("100us", 1e-4), ("0", 0.0)])
def test_go_durations(text, sec):
    assert parse_duration(text) == pytest.approx(sec)


@pytest.mark.parametrize("bad", ["", "5x", "s", "1s2"])
def test_bad_durations(bad):
    with pytest.raises(ValueError):
        parse_duration(bad)


def test_reference_config_surface_and_precedence(tmp_path):
    # the reference's key-declaration file: every key present with "" (.container/appconfig.yaml:1-10)
    (tmp_path / "appconfig.yaml").write_text("".join(f'{k}: ""\n' for k in REF_KEYS) + "workers: 3\n")
    (tmp_path / "appconfig.local.yaml").write_text("workers: 5\nalias: local-alias\n")
    env = {"APPLICATION_ENVIRONMENT": "local", "NEXUS__WORKERS": "10", "NEXUS__FAILURE_RATE_BASE_DELAY": "30ms",
           "NEXUS__FAILURE_RATE_MAX_DELAY": "5s", "NEXUS__RATE_LIMIT_ELEMENTS_PER_SECOND": "50",
           "NEXUS__RATE_LIMIT_ELEMENTS_BURST": "300", "NEXUS__CONTROLLER_NAMESPACE": "nexus",
           "NEXUS__LOG_LEVEL": "DEBUG", "NEXUS__SHARD_CONFIG_PATH": "./shards"}
    cfg = load_config(str(tmp_path), env)
    assert cfg.workers == 10 and cfg.alias == "local-alias"       # env > env-specific yaml > base yaml
    assert cfg.failure_rate_base_delay == pytest.approx(0.03) and cfg.failure_rate_max_delay == 5.0
    assert (cfg.rate_limit_elements_per_second, cfg.rate_limit_elements_burst) == (50, 300)
    assert cfg.controller_namespace == "nexus" and cfg.log_level == "DEBUG" and cfg.shard_config_path == "./shards"
    assert {AppConfig.key_of(a) for a in AppConfig.__dataclass_fields__} >= set(REF_KEYS)
    with pytest.raises(ValueError):
        load_config(str(tmp_path), {"NEXUS__WORKERS": "many"})


def test_config_roundtrips_through_env():
    cfg = AppConfig(workers=7, failure_rate_base_delay=0.25, mode="compat", transport="aiohttp")
    back = load_config("/nonexistent", config_to_env(cfg))
    assert back == cfg


def test_defaults_follow_helm_values():
    cfg = load_config("/nonexistent", {})
    assert (cfg.alias, cfg.shard_config_path, cfg.controller_namespace, cfg.workers) == \
        ("controller-cluster", "/app/config/shards", "nexus", 2)
    assert (cfg.failure_rate_base_delay, cfg.failure_rate_max_delay) == (0.03, 5.0)


def test_kubeconfig_variants(tmp_path):
    ca = b"-----BEGIN CERTIFICATE-----\nMIIB\n-----END CERTIFICATE-----\n"
    (tmp_path / "ca.crt").write_bytes(ca)
    (tmp_path / "token").write_text("file-token\n")
    doc = {
        "current-context": "b",
        "clusters": [{"name": "c1", "cluster": {"server": "https://a.example:6443/",
                                                "certificate-authority-data": base64.b64encode(ca).decode()}},
                     {"name": "c2", "cluster": {"server": "https://b.example", "certificate-authority": "ca.crt",
                                                "tls-server-name": "kube.b"}}],
        "users": [{"name": "u1", "user": {"token": "t1"}}, {"name": "u2", "user": {"tokenFile": "token"}}],
        "contexts": [{"name": "a", "context": {"cluster": "c1", "user": "u1"}},
                     {"name": "b", "context": {"cluster": "c2", "user": "u2", "namespace": "nexus"}}],
    }
    cfg = parse_kubeconfig(doc, base_dir=str(tmp_path))
    assert cfg.server == "https://b.example" and cfg.ca_data == ca and cfg.tls_server_name == "kube.b"
    assert cfg.token_file.endswith("token") and cfg.namespace == "nexus"
    a = parse_kubeconfig(doc, context="a")
    assert a.server == "https://a.example:6443" and a.token == "t1" and a.ca_data == ca
    with pytest.raises(ConfigError):
        parse_kubeconfig(doc, context="missing")


@pytest.mark.parametrize("http2", ["off", "on"])
async def test_exec_plugin_token_is_cached_and_refreshed(tmp_path, http2):
    counter = tmp_path / "count"
    script = tmp_path / "get-token"
    script.write_text(f"""#!{sys.executable}
import json, os, sys
p = {str(counter)!r}
n = int(open(p).read()) + 1 if os.path.exists(p) else 1
open(p, "w").write(str(n))
info = json.loads(os.environ["KUBERNETES_EXEC_INFO"])
assert info["kind"] == "ExecCredential"
print(json.dumps({{"apiVersion": "client.authentication.k8s.io/v1", "kind": "ExecCredential",
                  "status": {{"token": os.environ["TOKEN_PREFIX"] + str(n),
                             "expirationTimestamp": "2999-01-01T00:00:00Z"}}}}))
""")
    script.chmod(script.stat().st_mode | stat.S_IEXEC)
    kc = tmp_path / "shard.kubeconfig"
    kc.write_text(render_kubeconfig("http://127.0.0.1:1", "shard", exec_cfg={
        "apiVersion": "client.authentication.k8s.io/v1", "command": str(script), "args": [],
        "env": [{"name": "TOKEN_PREFIX", "value": "tok-"}], "provideClusterInfo": True}))
    cfg = load_kubeconfig(str(kc))
    creds = CredentialSource(cfg)
    assert await creds.token() == "tok-1"
    assert await creds.token() == "tok-1" and creds.exec_runs == 1      # cached until expiry
    assert await creds.token(force_refresh=True) == "tok-2"
    # a 401 from the apiserver triggers exactly one refresh and retry
    srv = FakeApiServer(token="tok-3")
    url = await srv.start()
    cfg.server = url
    client = RestClient(cfg, http2=http2)  # over HTTP/2 the authorization field is re-encoded with the new token
    try:
        client.creds._token = "tok-2"
        assert (await client.list(R.SECRETS, "nexus"))["items"] == []
        assert client.creds.exec_runs == 1 and counter.read_text() == "3"
        assert client.protocol == ("h2" if http2 == "on" else "http/1.1")
    finally:
        await client.close()
        await srv.stop()


def test_in_cluster_and_build_config(tmp_path, monkeypatch):
    monkeypatch.delenv("KUBERNETES_SERVICE_HOST", raising=False)
    with pytest.raises(ConfigError):
        in_cluster_config()
    monkeypatch.setenv("KUBERNETES_SERVICE_HOST", "10.0.0.1")
    monkeypatch.setenv("KUBERNETES_SERVICE_PORT", "443")
    cfg = build_config("")
    assert cfg.server == "https://10.0.0.1:443" and cfg.token_file.endswith("/token")
    kc = tmp_path / "c.kubeconfig"
    kc.write_text(render_kubeconfig("http://x:1", "c", token="t"))
    assert build_config(str(kc)).token == "t"


def test_shard_discovery_matches_secret_volume_layout(tmp_path):
    for n in ("kind-nexus-shard-0", "b-cluster", "a-cluster"):
        (tmp_path / f"{n}.kubeconfig").write_text("x")
    (tmp_path / "README").write_text("ignored")
    os.makedirs(tmp_path / "..2024_01_01", exist_ok=True)
    (tmp_path / "..data").symlink_to(tmp_path / "..2024_01_01")
    assert [n for n, _ in discover(str(tmp_path))] == ["a-cluster", "b-cluster", "kind-nexus-shard-0"]
    assert discover(str(tmp_path / "missing")) == []


async def test_bearer_token_via_rest_client_against_fake():
    srv = FakeApiServer(token="abc")
    url = await srv.start()
    try:
        ok = RestClient(ClusterConfig(server=url, token="abc"))
        assert (await ok.create(R.SECRETS, "nexus", {"metadata": {"name": "x"}, "data": {}}))["kind"] == "Secret"
        await ok.close()
        nok = RestClient(ClusterConfig(server=url, username="u", password="p"))
        with pytest.raises(E.Unauthorized):
            await nok.get(R.SECRETS, "nexus", "x")
        await nok.close()
    finally:
        await srv.stop()


def test_statsd_and_json_logging(capsys):
    import socket

    from ncc.telemetry.logging import configure_logging
    from ncc.telemetry.statsd import StatsdClient
    rx = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    rx.bind(("127.0.0.1", 0))
    rx.settimeout(2)
    c = StatsdClient("nexus_configuration_controller", f"udp://127.0.0.1:{rx.getsockname()[1]}", ["service:ncc"])
    c.gauge("workqueue_length", 3)
    c.gauge("workqueue_length", 5)          # aggregated: last value wins within a flush interval
    c.count("reconciles", 1, {"kind": "template"})
    c.count("reconciles", 2, {"kind": "template"})
    c.flush()
    assert rx.recv(1024) == (b"nexus_configuration_controller.workqueue_length:5|g|#service:ncc\n"
                             b"nexus_configuration_controller.reconciles:3|c|#service:ncc,kind:template")
    c.close()
    rx.close()
    import logging
    configure_logging("DEBUG", "json")
    logging.getLogger("ncc.test").info("hello", extra={"shard": "s0"})
    line = capsys.readouterr().out.strip().splitlines()[-1]
    rec = json.loads(line)
    assert rec["msg"] == "hello" and rec["shard"] == "s0" and rec["level"] == "INFO"
    configure_logging("WARNING", "text")


def test_helm_env_names_map_to_config_keys():
    """Every NEXUS__* variable the chart sets must be a real AppConfig key (no silently ignored settings)."""
    import re
    from dataclasses import fields
    from pathlib import Path
    tpl = (Path(__file__).parent.parent / "deploy/helm/nexus-configuration-controller/templates/deployment.yaml"
           ).read_text()
    names = set(re.findall(r"name: (NEXUS__[A-Z0-9_]+)", tpl))
    known = {AppConfig.env_of(f.name) for f in fields(AppConfig)}
    assert names and names <= known, names - known
    assert {"NEXUS__LEADER_ELECT", "NEXUS__SERVER_SIDE_APPLY", "NEXUS__WORKERS"} <= names


def test_cpu_share_reads_cgroup_quota(tmp_path):
    from ncc.app import auto_executors_per_shard, cgroup_cpu_quota
    (tmp_path / "cpu.max").write_text("1600000 100000\n")
    assert cgroup_cpu_quota(str(tmp_path)) == 16.0
    (tmp_path / "cpu.max").write_text("max 100000\n")
    assert cgroup_cpu_quota(str(tmp_path)) is None
    assert [auto_executors_per_shard(n, cpus=16) for n in (1, 2, 4, 8, 16)] == [4, 4, 4, 2, 1]
    assert auto_executors_per_shard(8, cpus=128) == 4 and auto_executors_per_shard(1, cpus=2) == 2


def test_shard_groups_capped_by_cpus():
    """One executor process per shard, no more than the CPUs (each holds its own controller-side cache)."""
    from ncc.app import auto_shard_groups
    assert [auto_shard_groups(n, cpus=16) for n in (1, 2, 8, 20)] == [1, 2, 8, 16]
    assert [auto_shard_groups(n, cpus=1) for n in (1, 8)] == [1, 1]
    assert auto_shard_groups(8, cpus=3) == 3


def test_cgroup_quota_of_own_cgroup(tmp_path):
    """A process placed in a sub-cgroup (v1 `cpu:/pods/x`, v2 `0::/pods/x`) reads its limit there, not at
    the unlimited mount root; in a pod's cgroup namespace (path "/") the mount root is its own cgroup."""
    from ncc.app import cgroup_cpu_quota
    root = tmp_path / "cg"
    (root / "cpu").mkdir(parents=True)
    (root / "cpu" / "cpu.cfs_quota_us").write_text("-1\n")
    (root / "cpu" / "cpu.cfs_period_us").write_text("100000\n")
    sub = root / "cpu" / "pods" / "x"
    sub.mkdir(parents=True)
    (sub / "cpu.cfs_quota_us").write_text("100000\n")
    (sub / "cpu.cfs_period_us").write_text("100000\n")
    proc = tmp_path / "cgroup"
    proc.write_text("4:memory:/pods/x\n1:cpu,cpuacct:/pods/x\n0::/\n")
    assert cgroup_cpu_quota(str(root), str(proc)) == 1.0
    proc.write_text("1:cpu,cpuacct:/\n0::/\n")
    assert cgroup_cpu_quota(str(root), str(proc)) is None
    v2 = tmp_path / "v2"
    (v2 / "pods" / "y").mkdir(parents=True)
    (v2 / "cpu.max").write_text("max 100000\n")
    (v2 / "pods" / "y" / "cpu.max").write_text("250000 100000\n")
    proc.write_text("0::/pods/y\n")
    assert cgroup_cpu_quota(str(v2), str(proc)) == 2.5


def test_klog_style_flags(monkeypatch, capsys):
    """main.go:36-37 — klog.InitFlags + flag.Parse: `-v=4` and klog's output flags are accepted, Go style."""
    import ncc.app as app
    from ncc.config import AppConfig
    assert app._go_style_flags(["-v=4", "-logtostderr", "--vmodule=x=2", "-v", "2"]) == \
        ["-v=4", "--logtostderr", "--vmodule=x=2", "-v", "2"]
    assert app.main(["-v=4", "-logtostderr=true", "--alsologtostderr", "-stderrthreshold", "INFO", "--version"]) == 0
    assert capsys.readouterr().out.strip() == app.__version__
    seen = {}

    async def fake_amain(cfg, control_fd=None):
        seen["level"] = cfg.log_level
        return 0
    monkeypatch.setattr(app, "_amain", fake_amain)
    monkeypatch.setattr(app, "load_config", lambda _d: AppConfig(log_level="INFO"))
    monkeypatch.setattr(app, "configure_logging", lambda *a, **k: None)
    assert app.main(["-v=4"]) == 0 and seen["level"] == "DEBUG"
    assert app.main(["-v", "2"]) == 0 and seen["level"] == "INFO"


def test_coalesce_window_key_reaches_native_options(monkeypatch):
    from ncc.app import options_from_config
    from ncc.config import AppConfig
    assert AppConfig().coalesce_window == 0.002
    monkeypatch.setenv("NEXUS__COALESCE_WINDOW", "7ms")
    from ncc.config import load_config
    cfg = load_config(None)
    assert cfg.coalesce_window == 0.007
    assert options_from_config(cfg).coalesce_window == 0.007
    cfg.mode = "compat"
    assert options_from_config(cfg).coalesce_window == 0.0  # reference: every event enqueues at once


def test_native_workers_floor():
    from ncc.app import options_from_config
    from ncc.config import AppConfig
    cfg = AppConfig(mode="native")  # reference default workers=2
    assert options_from_config(cfg).workers == 32
    cfg.workers = 64
    assert options_from_config(cfg).workers == 64
    cfg.native_workers, cfg.workers = 8, 2
    assert options_from_config(cfg).workers == 8
    assert options_from_config(AppConfig(mode="compat")).workers == 2  # reference semantics


def test_coordinator_partition_rules(monkeypatch):
    from ncc.app import auto_coordinator_partitions, coordinator_partition
    from ncc.config import AppConfig
    assert auto_coordinator_partitions(2, 3, cpus=256) == 1        # few shards: one coordinator
    assert auto_coordinator_partitions(8, 3, cpus=16) == 1         # the 16-CPU box: CPU-bound anyway
    assert auto_coordinator_partitions(8, 3, cpus=64) == 1         # C must divide k: not enough CPUs for 3
    assert auto_coordinator_partitions(8, 3, cpus=128) == 3        # one coordinator per executor partition
    assert auto_coordinator_partitions(8, 2, cpus=256) == 2
    monkeypatch.delenv("NCC_COORDINATOR_PART", raising=False)
    assert coordinator_partition(AppConfig(coordinator_partitions=1), 8, 3) is None
    assert coordinator_partition(AppConfig(coordinator_partitions=3), 1, 1) == (0, 3)
    monkeypatch.setenv("NCC_COORDINATOR_PART", "2/3")
    assert coordinator_partition(AppConfig(coordinator_partitions=1), 8, 3) == (2, 3)  # a child


def test_executor_pool_global_partitions():
    from ncc.controller.executor import ExecutorPool, key_part
    pool = ExecutorPool(["s0", "s1"], 2, lambda i, m: None, per_shard=2, part_base=1, part_stride=3)
    assert [(h.shards, h.part, h.parts) for h in pool.handles] == \
        [(["s0"], 1, 6), (["s0"], 4, 6), (["s1"], 1, 6), (["s1"], 4, 6)]
    # every key of executor partition q of 6 belongs to coordinator partition q % 3
    for i in range(200):
        k = f"template/nexus/algo-{i:05d}"
        assert key_part(k, 6) % 3 == key_part(k, 3)


def test_native_auto_sizing_and_cpu_override(monkeypatch):
    """Native executors: one per shard; coordinator processes one per 32 CPUs (≤ 4) from 4 shards up.
    NCC_CPU_SHARE rehearses a large host's sizing on a small one."""
    from ncc.app import auto_sizing, cpu_share
    assert auto_sizing(1, cpus=16, native=True) == (1, 1)
    assert auto_sizing(4, cpus=16, native=True) == (1, 1)
    assert auto_sizing(8, cpus=64, native=True) == (1, 2)
    assert auto_sizing(8, cpus=128, native=True) == (1, 2)  # one coordinator per 4 shard groups
    assert auto_sizing(4, cpus=512, native=True) == (1, 1)
    assert auto_sizing(8, cpus=512, native=True) == (1, 2)
    assert auto_sizing(16, cpus=512, native=True) == (1, 4)
    assert auto_sizing(32, cpus=24, native=True) == (1, 3)  # capped by 8 CPUs per coordinator
    assert auto_sizing(8, cpus=16, native=True) == (1, 2) and auto_sizing(8, cpus=8, native=True) == (1, 1)
    assert auto_sizing(8, cpus=128, native=False) == (4, 4)  # Python executors: k = C = 4
    monkeypatch.setenv("NCC_CPU_SHARE", "128")
    assert cpu_share() == 128


def test_nofile_limit_raised_to_hard(monkeypatch):
    """Every ncc process lifts its soft RLIMIT_NOFILE to the hard limit (as the Go runtime does)."""
    import resource

    from ncc.proclimits import raise_nofile_limit
    calls = []
    monkeypatch.setattr(resource, "getrlimit", lambda r: (1024, 65536))
    monkeypatch.setattr(resource, "setrlimit", lambda r, v: calls.append(v))
    assert raise_nofile_limit() == 65536 and calls == [(65536, 65536)]
    monkeypatch.setattr(resource, "getrlimit", lambda r: (65536, 65536))
    calls.clear()
    assert raise_nofile_limit() == 65536 and calls == []
