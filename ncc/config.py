"""Application configuration: `appconfig.yaml` + `appconfig.<env>.yaml` + `NEXUS__*` environment.

Reference contract:
* typed target `AppConfig` with ten keys (pkg/models/app_config.go:21-32);
* nexus-core `LoadConfig[T]` reads `appconfig.yaml`, overlays `appconfig.<APPLICATION_ENVIRONMENT>.yaml`
  (CI sets `local`, build.yaml:79), then environment overrides with the `NEXUS__` prefix where the
  key's `-` becomes `_` and the name is upper-cased (deployment.yaml:50-69, build.yaml:68-79);
* durations are Go duration strings (`30ms`, `5s`, `1m30s`).
The YAML files list every key with `""` (.container/appconfig.yaml:1-10): an empty value means
"not set here".  Unset keys take the Helm chart's defaults (values.yaml:135-169) rather than
Go zero values, so a bare `python -m ncc` is usable.

Extra keys of this framework (all optional, same env convention): `mode`, `client-qps`,
`client-burst`, `client-pool-size`, `client-pipeline-depth`, `client-http2`, `transport`, `server-side-apply`, `sync-dependent-metadata`, `controller-adoption`, `executors`, `max-executors`, `executors-per-shard`, `resync-period`, `full-resync-period`, `shard-sync-timeout`, `shard-reload-period`, `coalesce-window`, `event-repeat-window`, `native-workers`, `coordinator-partitions`, `watch-relay`, `executor-impl`,
`metrics-bind-address`, `health-bind-address`, `log-format`, `leader-elect`,
`leader-election-namespace`, `leader-election-lease-name`, `lease-duration`, `renew-deadline`, `retry-period`.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field, fields

import yaml

ENV_PREFIX = "NEXUS__"

_DUR_RE = re.compile(r"([0-9]*\.?[0-9]+)(ns|us|µs|μs|ms|s|m|h)")
_UNITS = {"ns": 1e-9, "us": 1e-6, "µs": 1e-6, "μs": 1e-6, "ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}


def parse_duration(v) -> float:
    """Go `time.ParseDuration` → seconds.  Bare numbers are taken as seconds."""
    if isinstance(v, (int, float)):
        return float(v)
    s = str(v).strip()
    if not s:
        raise ValueError("empty duration")
    sign = 1.0
    if s[0] in "+-":
        sign = -1.0 if s[0] == "-" else 1.0
        s = s[1:]
    if s == "0":
        return 0.0
    try:
        return sign * float(s)
    except ValueError:
        pass
    pos, total = 0, 0.0
    for m in _DUR_RE.finditer(s):
        if m.start() != pos:
            raise ValueError(f"invalid duration {v!r}")
        total += float(m.group(1)) * _UNITS[m.group(2)]
        pos = m.end()
    if pos != len(s):
        raise ValueError(f"invalid duration {v!r}")
    return sign * total


def _dur(default: float):
    return field(default=default, metadata={"type": "duration"})


@dataclass
class AppConfig:
    # ---- the reference's ten keys (pkg/models/app_config.go:22-31) ----
    alias: str = "controller-cluster"
    controller_config_path: str = ""
    shard_config_path: str = "/app/config/shards"
    controller_namespace: str = "nexus"
    log_level: str = "INFO"
    workers: int = 2
    native_workers: int = 32         # native: reconcile workers per process (coordinator, each executor);
                                     # `workers` raises it when larger (box sweep: 16–32 best, 64 worse)
    failure_rate_base_delay: float = _dur(0.030)
    failure_rate_max_delay: float = _dur(5.0)
    rate_limit_elements_per_second: int = 50
    rate_limit_elements_burst: int = 300
    # ---- framework extensions ----
    mode: str = "native"
    client_qps: float = 0.0          # 0 = mode default (compat: client-go's 5/10, native: none); < 0 = none
    client_burst: int = 10
    client_pool_size: int = 0        # keep-alive connections per cluster; 0 = auto: 64 for the Python clients,
                                     # 256 for the C++ executor's shard clients
    client_pipeline_depth: int = 0   # HTTP/1.1-pipelined requests per connection (in flight ≤ pool × depth);
                                     # 0 = auto: 1 (no pipelining)
    client_http2: str = "auto"       # every client (controller cluster and shards): auto (HTTP/2 where TLS
                                     # negotiates it by ALPN, as client-go) | on (also prior-knowledge HTTP/2 on
                                     # cleartext shards; see controller_http2) | off
    transport: str = "fast"          # fast (raw asyncio HTTP/1.1) | aiohttp
    server_side_apply: bool = False  # native mode: write shard objects with server-side apply
    sync_dependent_metadata: bool = False  # native mode: shard Secrets/ConfigMaps carry the source's labels
                                           # and annotations (plus the owner labels)
    controller_adoption: bool = True  # add template ownerRefs to controller-side Secrets/ConfigMaps (reference)
    executors: int = -1              # shard-executor processes; -1 = auto (native: one per shard, ≤ max)
    max_executors: int = 16
    executors_per_shard: int = -1    # key-partitioned executors per shard group; -1 = auto (app.py)
    coordinator_partitions: int = -1  # native: coordinator processes splitting the template keys; -1 = auto
    executor_impl: str = "auto"      # native: shard executors as ncc/bin/ncc-executor (C++) when built and
                                     # supported ("auto"), always "native", or "python"
    watch_relay: bool = True         # native: executors get the controller cluster from the coordinator's
                                     # LIST/WATCH (ncc/controller/relay.py) instead of their own
    resync_period: float = _dur(30.0)
    full_resync_period: float = _dur(600.0)
    shard_sync_timeout: float = _dur(10.0)
    shard_reload_period: float = _dur(30.0)  # native: re-scan shard-config-path for added/removed/changed shards
    coalesce_window: float = _dur(0.002)  # native: park event-triggered keys this long so a template and its
                                          # Secret/ConfigMap changing together reconcile once
    event_repeat_window: float = _dur(1.0)  # native: repeats of an Event already written are folded into one
                                            # count PATCH per window (first occurrences go out at once)
    metrics_bind_address: str = ""   # e.g. ":9090" → Prometheus /metrics
    health_bind_address: str = ""    # e.g. ":8081" → /healthz, /readyz
    log_format: str = "json"
    leader_elect: bool = False       # Lease-based leader election (run >1 replica; ncc/leader.py)
    leader_election_namespace: str = ""   # default: controller-namespace
    leader_election_lease_name: str = "nexus-configuration-controller"
    lease_duration: float = _dur(15.0)
    renew_deadline: float = _dur(10.0)
    retry_period: float = _dur(2.0)

    def pool_size(self) -> int:
        """client-pool-size for the Python transport (0 = its default of 64)."""
        return self.client_pool_size if self.client_pool_size > 0 else 64

    def pipeline_depth(self) -> int:
        """client-pipeline-depth for the Python transport (0 = its default of 1: no pipelining)."""
        return self.client_pipeline_depth if self.client_pipeline_depth > 0 else 1

    @staticmethod
    def key_of(attr: str) -> str:
        return attr.replace("_", "-")

    @staticmethod
    def env_of(attr: str) -> str:
        return ENV_PREFIX + attr.upper()


def _coerce(f, raw):
    if f.metadata.get("type") == "duration":
        return parse_duration(raw)
    t = f.type if isinstance(f.type, str) else getattr(f.type, "__name__", str(f.type))
    if t == "int":
        return int(float(raw))
    if t == "float":
        return float(raw)
    if t == "bool":
        return str(raw).lower() in ("1", "true", "yes", "on")
    return str(raw)


def _read_yaml(path: str) -> dict:
    if not os.path.exists(path):
        return {}
    with open(path) as fh:
        return yaml.safe_load(fh) or {}


HTTP2_MODES = {"off": 0, "auto": 1, "on": 2}  # client-http2 -> the C++ executor's `http2` (native/executor/http.hpp)


def controller_http2(mode: str) -> str:
    """The controller cluster's client negotiates HTTP/2 as client-go does — by ALPN on TLS — whatever
    `client-http2` says: `on` adds prior knowledge on cleartext for the shard clients only.  Measured on the
    bench's cleartext apiservers (profiles/r5/r5k, r5m: 5 pairs), prior-knowledge HTTP/2 to the controller
    apiserver cost 2-13 % objects/s; over TLS, where it is negotiated, it saves coordinator CPU."""
    return "auto" if mode == "on" else mode


def load_config(config_dir: str | None = None, env: dict | None = None) -> AppConfig:
    env = os.environ if env is None else env
    config_dir = config_dir or env.get("NCC_CONFIG_DIR") or os.getcwd()
    merged: dict = {}
    merged.update(_read_yaml(os.path.join(config_dir, "appconfig.yaml")))
    app_env = env.get("APPLICATION_ENVIRONMENT")
    if app_env:
        merged.update(_read_yaml(os.path.join(config_dir, f"appconfig.{app_env}.yaml")))
    cfg = AppConfig()
    for f in fields(AppConfig):
        raw = merged.get(AppConfig.key_of(f.name))
        ev = env.get(AppConfig.env_of(f.name))
        if ev not in (None, ""):
            raw = ev
        if raw is None or raw == "":
            continue
        try:
            v = _coerce(f, raw)
            if f.name == "client_http2":
                v = str(v).strip().lower()
                if v not in HTTP2_MODES:
                    raise ValueError(f"one of {', '.join(HTTP2_MODES)}")
            setattr(cfg, f.name, v)
        except ValueError as e:
            raise ValueError(f"invalid value for {AppConfig.key_of(f.name)}: {raw!r} ({e})") from e
    return cfg


def config_to_env(cfg: AppConfig) -> dict:
    """Render a config as NEXUS__* variables (how the coordinator hands its config to executors)."""
    out = {}
    for f in fields(AppConfig):
        v = getattr(cfg, f.name)
        out[AppConfig.env_of(f.name)] = repr(v) if isinstance(v, float) else str(v)
    return out
