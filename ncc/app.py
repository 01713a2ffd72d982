"""Process entry point: `python -m ncc` (reference `main()`, main.go:35-109).

Boot sequence, as in the reference:
  signals → config → logger + statsd → controller-cluster client → namespace-scoped informers
  (resync 30 s) → shards from the kubeconfig directory (informers started) → controller →
  start controller informers → `controller.run()` until SIGTERM/SIGINT.
A setup error exits with status 1 (`klog.FlushAndExit`).  Unlike the reference
(main.go:97-103) the controller is built *before* anything is started, so a construction
error cannot leave informers running.

`mode=compat` reproduces the reference's runtime semantics including client-go's default
client-side QPS (5/burst 10 per API group) — used for baseline measurements;
`mode=native` (default) enables the improvements in `ControllerOptions.native()`.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import signal
import sys

from . import __version__, gctune, loopmon
from . import native as native_ext
from .api import constants as C
from .api import resources as R
from .cache.informer import InformerFactory
from .config import AppConfig, config_to_env, controller_http2, load_config
from .controller.controller import Controller
from .controller.events import BroadcastRecorder, FakeRecorder
from .controller.executor import CoordinatorPartitions, ExecutorPool, partition_filter, partition_owner_filter
from .controller.options import ControllerOptions
from .kube.client import RateLimitedClient
from .kube.kubeconfig import build_config
from .kube.rest import RestClient
from .leader import LeaderElector, identity_from_env
from .shards.loader import default_client_factory, discover, load_shards
from .telemetry.logging import configure_logging
from .telemetry.statsd import MultiMetrics, StatsdClient

log = logging.getLogger("ncc")

COMPAT_QPS, COMPAT_BURST = 5.0, 10  # client-go rest.DefaultQPS / DefaultBurst


def options_from_config(cfg: AppConfig) -> ControllerOptions:
    kw = dict(workers=cfg.workers, failure_base_delay=cfg.failure_rate_base_delay,
              failure_max_delay=cfg.failure_rate_max_delay, rate_limit_qps=float(cfg.rate_limit_elements_per_second),
              rate_limit_burst=cfg.rate_limit_elements_burst, resync_period=cfg.resync_period)
    if cfg.mode == "native":
        # the reference's `workers` (Helm default 2) sized sequential Go reconciles; a native process hides
        # shard RTTs behind cheap coroutines, so it runs at least `native-workers`
        kw["workers"] = max(cfg.workers, cfg.native_workers)
        kw.update(full_resync_period=cfg.full_resync_period, wait_for_shards_timeout=cfg.shard_sync_timeout,
                  server_side_apply=cfg.server_side_apply, controller_adoption=cfg.controller_adoption,
                  sync_dependent_metadata=cfg.sync_dependent_metadata,
                  coalesce_window=cfg.coalesce_window)
    opts = ControllerOptions.for_mode(cfg.mode, **kw)
    # expert/ablation overrides: NCC_OPT_<FIELD>=value (e.g. NCC_OPT_COALESCE_WINDOW=0)
    for f, cur in opts.as_dict().items():
        raw = os.environ.get("NCC_OPT_" + f.upper())
        if raw is None:
            continue
        if isinstance(cur, bool) or cur is None and raw.lower() in ("true", "false"):
            val = raw.lower() in ("1", "true", "yes")
        elif isinstance(cur, int):
            val = int(raw)
        elif isinstance(cur, float) or cur is None:
            val = float(raw)
        else:
            val = raw
        setattr(opts, f, val)
    return opts


def client_limits(cfg: AppConfig) -> tuple[float, int]:
    """(qps, burst) of the client-side token bucket; qps 0 = no limiter.  `client-qps` > 0 sets it,
    < 0 switches it off in every mode (the "compat-unthrottled" baseline: reference scheduling without
    client-go's default 5 QPS / burst 10), 0 keeps the mode default."""
    if cfg.client_qps > 0:
        return cfg.client_qps, cfg.client_burst
    if cfg.client_qps < 0:
        return 0.0, cfg.client_burst
    if cfg.mode == "compat":
        return COMPAT_QPS, COMPAT_BURST
    return 0.0, cfg.client_burst


def shard_files(path: str) -> dict:
    """{shard name: sha256 of its kubeconfig} for the shard config directory."""
    import hashlib
    out = {}
    for name, p in discover(path):
        try:
            with open(p, "rb") as f:
                out[name] = hashlib.sha256(f.read()).hexdigest()
        except OSError:
            continue
    return out


def strip_payload(obj: dict) -> dict:
    """The coordinator's stored form of a Secret/ConfigMap: no payload, and no metadata.managedFields (server-side
    apply's field ownership: hundreds of bytes per object on a real apiserver, never read here)."""
    out = {k: v for k, v in obj.items() if k not in ("data", "binaryData", "stringData")}
    m = out.get("metadata")
    if isinstance(m, dict) and "managedFields" in m:
        out["metadata"] = {k: v for k, v in m.items() if k != "managedFields"}
    return out


def own_cgroups(proc_file: str = "/proc/self/cgroup") -> dict:
    """{controller: path} of this process's cgroups ("" = the v2 unified hierarchy).  Inside a pod (a cgroup
    namespace) every path is "/"; a process placed in a sub-cgroup (a sidecar-less limit, or bench/suite.py's
    `--cgroup`) sees its own path here, and its limit lives there, not at the mount root."""
    out = {}
    try:
        with open(proc_file) as f:
            for line in f:
                _, ctrls, path = line.rstrip("\n").split(":", 2)
                for c in (ctrls.split(",") if ctrls else [""]):
                    out[c] = path
    except (OSError, ValueError):
        pass
    return out


def _cgroup_dirs(root: str, v1_controller: str, proc_file: str) -> list:
    """Candidate directories of this process's cgroup for one v1 controller (and the v2 hierarchy), most
    specific first, ending at the mount roots."""
    mine = own_cgroups(proc_file)
    dirs = []
    for base, key in ((os.path.join(root, v1_controller), v1_controller), (root, ""),
                      (os.path.join(root, "unified"), "")):
        p = mine.get(key)
        if p and p != "/":
            dirs.append(os.path.join(base, p.lstrip("/")))
        dirs.append(base)
    return dirs


def cgroup_cpu_quota(root: str = "/sys/fs/cgroup", proc_file: str = "/proc/self/cgroup") -> float | None:
    """CPU limit from the cgroup CFS quota (v2 `cpu.max`, v1 `cpu.cfs_quota_us`), None if unlimited.
    A Kubernetes pod's `resources.limits.cpu` lands here, not in the affinity mask.  The process's own cgroup
    (/proc/self/cgroup) is read first, then the mount root (a pod's cgroup namespace puts its cgroup there)."""
    for d in _cgroup_dirs(root, "cpu", proc_file):
        try:
            with open(os.path.join(d, "cpu.max")) as f:
                quota, _, period = f.read().strip().partition(" ")
            if quota != "max":
                return int(quota) / int(period or 100000)
            return None
        except (OSError, ValueError):
            pass
        try:
            with open(os.path.join(d, "cpu.cfs_quota_us")) as f:
                quota = int(f.read().strip())
            with open(os.path.join(d, "cpu.cfs_period_us")) as f:
                period = int(f.read().strip())
            return quota / period if quota > 0 and period > 0 else None
        except (OSError, ValueError):
            continue
    return None


def cpu_share() -> int:
    """CPUs this process may really use: the affinity mask capped by the cgroup CPU quota.
    `NCC_CPU_SHARE=<n>` overrides it (rehearsing a large host's automatic sizing on a small one)."""
    forced = os.environ.get("NCC_CPU_SHARE")
    if forced:
        return max(1, int(forced))
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):  # pragma: no cover - non-Linux
        n = os.cpu_count() or 1
    q = cgroup_cpu_quota()
    return max(1, min(n, int(q))) if q else n


def auto_shard_groups(shards: int, cpus: int | None = None) -> int:
    """Shard-executor processes (`executors: -1`): one per shard, but no more than the CPUs the pod may use.

    Each executor process holds its own copy of the controller-side objects its shards need (fed by the watch
    relay), so a process per shard costs memory in proportion; under a CPU quota smaller than the shard count
    the extra processes cannot run in parallel anyway.  At BASELINE config 4 (8 shards × 10 000 templates,
    bench/suite.py) one process for all 8 shards settled at 822 MiB for the whole controller against 1 517 MiB
    with eight (BENCHMARKS.md "Config 4 at scale")."""
    cpus = cpu_share() if cpus is None else cpus
    return max(1, min(shards, cpus))


def auto_executors_per_shard(groups: int, cpus: int | None = None) -> int:
    """Key-partitioned executors per shard group: one per CPU share of the group, 1..4.

    Measured on the MI355X host under a 16-CPU quota, 3 runs each (profiles/r1/session2/kgrid_rep/):
    N=1 k=3/4/5 25.2k/26.4k/26.8k, N=2 41.8k/46.1k/41.9k, N=4 72.4k/71.0k/74.8k objects/s, with p50 latency
    falling as k grows.  Since other partitions' lines are dropped natively before decoding, an extra
    executor costs little; past 4 the gain is within noise (the previous round's tree, which decoded every
    controller-side dependent in every executor, peaked at k=3: profiles/r1/kscan)."""
    import math
    cpus = cpu_share() if cpus is None else cpus
    return max(1, min(4, math.ceil(cpus / max(1, groups))))


def auto_coordinator_partitions(groups: int, per_shard: int, cpus: int | None = None) -> int:
    """Coordinator processes (Python executors): one per executor key partition (C = k) once there are ≥ 4
    shard groups and ≥ 32 CPUs per coordinator; otherwise one.  The coordinators share the k executors.  At 8 shards
    one coordinator spends ~210 µs per template pass on the box (profiles/r1/session2/spr_8.json), which caps
    a single process near 110k objects/s; on a CPU-bound host extra processes only cost
    (profiles/r1/session2/coord_partitions_*)."""
    cpus = cpu_share() if cpus is None else cpus
    if groups < 4 or per_shard < 2 or cpus // 32 < per_shard:
        return 1
    return per_shard


def auto_sizing(groups: int, cpus: int | None = None, native: bool = False) -> tuple[int, int]:
    """(executors per shard k, coordinator processes C) chosen automatically for `groups` shard groups.

    Python executors: k = one per CPU share of a group (1..4), C = k once there are ≥ 4 groups and
    ≥ 32 CPUs per coordinator (see the two functions above).

    Native executors (ncc/bin/ncc-executor): k = 1.  One C++ process per shard costs ~24 µs of CPU per
    synced object on the MI355X host and keeps up with a shard apiserver on its own
    (profiles/r2/native_executor_box/: k=1 28.2k objects/s at 52 µs/object in total vs k=4 28.8k at
    73 µs); extra partitions would only re-parse the same shard watch streams.

    The coordinator carries the per-template work (status, adoption, Events, reports).  One process keeps
    up with ~140-160k objects/s whether it serves 4 or 8 shards (box: N=4 134k at 0.93 cores,
    profiles/r2/sweep_r2e/; 8 shards on one rank 159k at 0.94 cores, profiles/r2/prof8/), i.e. with about
    4 shards at a shard apiserver's ~36k objects/s.  The partitions share the executors, so they cost the
    shards next to nothing (profiles/r2/c_on_one_shard_shared/); they cost CPU.  So C = one per 4 shard
    groups (N=8: 2), with 8 CPUs per coordinator, up to 4: 8 shards on one rank of the 16-CPU box ran
    141k/179k objects/s at C=1, 156k/214k at C=2, 150k/197k at C=4 (profiles/r2/spr8_c_shared/)."""
    import math
    cpus = cpu_share() if cpus is None else cpus
    if not native:
        k = auto_executors_per_shard(groups, cpus)
        return k, auto_coordinator_partitions(groups, k, cpus)
    if groups < 4:
        return 1, 1
    return 1, max(1, min(4, cpus // 8, math.ceil(groups / 4)))


def coordinator_partition(cfg: AppConfig, groups: int, per_shard: int, native: bool = False) -> tuple | None:
    """(p, C) for this coordinator process, or None when the coordinator is not split."""
    env = os.environ.get("NCC_COORDINATOR_PART")
    if env:  # a child started by CoordinatorPartitions
        pi, _, pk = env.partition("/")
        p, c = int(pi), int(pk)
        return (p, c) if c > 1 else None
    if cfg.coordinator_partitions > 0:
        c = cfg.coordinator_partitions
    elif native:
        c = auto_sizing(groups, native=True)[1]
    else:
        c = auto_coordinator_partitions(groups, per_shard)
    return (0, c) if c > 1 else None


class App:
    """Wires and owns every component of one controller process."""

    def __init__(self, cfg: AppConfig, *, client_factory=None, controller_client=None, metrics=None,
                 options: ControllerOptions | None = None, role: str | None = None, shard_filter: set | None = None):
        self.cfg = cfg
        self.options = options or options_from_config(cfg)
        if role is not None:
            self.options.role = role
        self.shard_filter = shard_filter
        self.pool: ExecutorPool | None = None
        self.n_executors = 0
        self.per_shard = 1
        qps, burst = client_limits(cfg)
        self.client_factory = client_factory or default_client_factory(qps, burst, cfg.pool_size(),
                                                                       cfg.transport, cfg.pipeline_depth(),
                                                                       cfg.client_http2)
        self._controller_client = controller_client
        self.metrics = metrics
        self.ops = None
        self.controller: Controller | None = None
        self.elector: LeaderElector | None = None
        self._lease_task = None
        self._reload_task = None
        self._gc_task = None
        self._lag_task = None
        self._shard_files: dict = {}
        self.lost_leadership = False
        self.gate: asyncio.Event | None = None  # workers wait for it (warm standby / pre-spawned child)
        self.relay = None  # coordinator: WatchRelay feeding the executors
        self.executor_impl = ""  # coordinator: "native" (ncc/bin/ncc-executor) or "python" shard executors
        self.executor_fallback = ""  # coordinator: why the Python executors run instead of the C++ ones ("" = they don't)
        self.cpu_affinity = ""  # coordinator: "l3:<cpus>" when it restricted itself to one L3 domain, else "none"
        self.placement = None  # coordinator with NCC_CPU_AFFINITY=l3: ncc.affinity.Placement
        self._placement_task = None
        self._cred_task = None
        self.native_cfg = None  # coordinator with C++ executors: NativeExecutorConfig (renders their config)
        self._relay_ok = False  # coordinator: the watch relay can run (decided once, in build)
        self.relay_feeds: list | None = None  # executor: per-kind feeds from the coordinator's relay
        self.standby_was_warm = False  # caches had synced before this replica acquired the Lease
        self.coord_part: tuple | None = None  # (p, C) when the coordinator role is split over C processes
        self.partitions: CoordinatorPartitions | None = None  # children for partitions 1..C-1 (parent only)

    async def build(self) -> Controller:
        cfg, o = self.cfg, self.options
        prom = None
        if self.metrics is None:
            sinks = [StatsdClient(C.METRIC_NAMESPACE)]
            if cfg.metrics_bind_address:
                from .telemetry.http import PrometheusMetrics
                prom = PrometheusMetrics(C.METRIC_NAMESPACE)
                sinks.append(prom)
            self.metrics = MultiMetrics(*sinks)
        client = self._controller_client
        if client is None:
            qps, burst = client_limits(cfg)
            client = RestClient(build_config(cfg.controller_config_path), pool_size=cfg.pool_size(),
                                pipeline_depth=cfg.pipeline_depth(), http2=controller_http2(cfg.client_http2),
                                cluster_name=cfg.alias, transport=cfg.transport)
            if qps > 0:
                client = RateLimitedClient(client, qps, burst)
        self.client = client
        # the watch relay needs the native extension and a transport that hands out raw watch lines: decided
        # here, once, for both the sizing below and the choice of executor implementation
        self._relay_ok = bool(cfg.watch_relay) and native_ext.load() is not None and hasattr(client, "watch_raw")
        self.factory = InformerFactory(client, cfg.controller_namespace, o.resync_period)
        all_names = [n for n, _ in discover(cfg.shard_config_path)]
        self._shard_files = shard_files(cfg.shard_config_path)
        if o.role == "all" and o.mode == "native" and all_names:
            n = cfg.executors if cfg.executors >= 0 else auto_shard_groups(len(all_names))
            self.n_executors = max(0, min(n, cfg.max_executors, len(all_names)))
            if self.n_executors > 0:
                o.role = "coordinator"
                from .controller.native_executor import choose
                native = choose(cfg, o, relay_active=self._relay_ok, quiet=True)[0]
                self.per_shard = (cfg.executors_per_shard if cfg.executors_per_shard > 0
                                  else auto_sizing(self.n_executors, native=native)[0])
                self.coord_part = coordinator_partition(cfg, self.n_executors, self.per_shard, native)
                if self.coord_part is not None:
                    o.partition = self.coord_part  # this coordinator's share of the template keys
                    if os.environ.get("NCC_COORDINATOR_PART"):
                        # a child: the parent's executors serve every key; it relays this partition's reports
                        self.n_executors = 0
        if o.role == "coordinator" and self.n_executors > 0 and (self.coord_part or (0, 1))[0] == 0:
            # NCC_CPU_AFFINITY=l3: the coordinator and its executors (and child partitions) on one L3 domain,
            # chosen here — before anything is spawned (children inherit the mask) and off the propagation path
            from . import affinity
            parts = (self.coord_part or (0, 1))[1]
            self.placement = await affinity.apply_async(1 + self.n_executors * max(1, self.per_shard) + parts - 1)
            self.cpu_affinity = f"l3:{len(self.placement.cpus)}" if self.placement else "none"
        kf = partition_filter(*o.partition) if o.partition is not None else None
        infs = {rt: self.factory.informer(rt, key_filter=kf if rt in (R.TEMPLATES, R.WORKGROUPS) else None)
                for rt in (R.SECRETS, R.CONFIGMAPS, R.TEMPLATES, R.WORKGROUPS)}
        if o.partition is not None and o.controller_adoption:
            # controller-side Secrets/ConfigMaps owned only by other partitions' templates are dropped before
            # decoding (adoption stamps every referenced dependent with its templates); one that a template
            # of this partition references but which is not (yet) owned by it is kept through the reverse index
            tstore = infs[R.TEMPLATES].store
            for rt, index in ((R.SECRETS, "secret"), (R.CONFIGMAPS, "configmap")):
                infs[rt].owner_filter = partition_owner_filter(
                    *o.partition, referenced=lambda ns, name, i=index: bool(tstore.by_index(i, f"{ns}/{name}")))
        if o.role == "executor" and os.environ.get("NCC_RELAY") == "1":
            # the coordinator lists and watches the controller cluster for us (ncc/controller/relay.py)
            from .controller.relay import KINDS, RelayFeed
            self.relay_feeds = []
            for rt in KINDS:
                infs[rt].feed = RelayFeed()
                self.relay_feeds.append(infs[rt].feed)
        if o.role == "coordinator":
            self.shards = []
            # the coordinator adopts and reports; it never copies payloads: keep metadata only and skip
            # payload-only updates straight off the wire
            for rt in (R.SECRETS, R.CONFIGMAPS):
                infs[rt].metadata_only = True
                infs[rt].store.transform = strip_payload
            # ...nor template specs beyond their references: templates arrive slim (metadata, status, the
            # Secret/ConfigMap references and a digest of the spec; `_native.template_event_slim`)
            mod = native_ext.load()
            if mod is not None and os.environ.get("NCC_SLIM_TEMPLATES") != "0":
                infs[R.TEMPLATES].slim_decode = mod.template_event_slim
        else:
            self.shards = load_shards(cfg.alias, cfg.shard_config_path, cfg.controller_namespace,
                                      client_factory=self.client_factory,
                                      resync_period=0.0 if o.watch_shards else o.resync_period,
                                      assume_writes=o.assume_writes, sync_binary_data=o.sync_binary_data,
                                      sync_metadata=o.sync_dependent_metadata,
                                      slim=o.slim_shard_cache, start=False, names=self.shard_filter,
                                      key_filter=kf, owner_filter=self._shard_owner_filter(infs))
        if o.role == "executor":
            self.recorder = FakeRecorder(keep=False)  # executors never write to the controller cluster
        else:
            # native: 4 writer tasks (per-object order kept) so Event traffic keeps up with fan-out rates;
            # compat: client-go's single sink goroutine
            native_events = o.mode == "native" and os.environ.get("NCC_EVENT_COALESCE") != "0"
            tstore, wstore = infs[R.TEMPLATES].store, infs[R.WORKGROUPS].store
            self.recorder = BroadcastRecorder(client, log_events=log.isEnabledFor(logging.DEBUG),
                                              writers=4 if o.mode == "native" else 1, coalesce=native_events,
                                              repeat_window=cfg.event_repeat_window if native_events else 0.0,
                                              cache_limit=(lambda: 2 * (len(tstore) + len(wstore)))
                                              if o.mode == "native" else 4096)
        self.controller = Controller(alias=cfg.alias, namespace=cfg.controller_namespace, client=client,
                                     shards=self.shards, template_informer=infs[R.TEMPLATES],
                                     workgroup_informer=infs[R.WORKGROUPS], secret_informer=infs[R.SECRETS],
                                     configmap_informer=infs[R.CONFIGMAPS], options=o, recorder=self.recorder,
                                     metrics=self.metrics,
                                     shard_names=all_names if o.role == "coordinator" else None)
        if cfg.metrics_bind_address or cfg.health_bind_address:
            from .telemetry.http import OpsServer
            self.ops = OpsServer(ready=self._ready,
                                 prometheus=prom, extra=self.debug_state, checks=self._ready_checks)
        if cfg.mode == "native":
            # start-up garbage (imports, config parsing) collected and the survivors frozen now, before any
            # informer or executor runs: a full pass over a large heap here is off the propagation path
            gctune.collect_startup()
        return self.controller

    async def reload_shards(self) -> dict:
        """Re-scan the shard kubeconfig directory and apply additions, removals and credential changes
        without a restart (the reference loads shards once at startup, main.go:73).  Returns the diff."""
        cfg, ctl = self.cfg, self.controller
        now = shard_files(cfg.shard_config_path)
        if self.shard_filter is not None:
            now = {n: h for n, h in now.items() if n in self.shard_filter}
        old = self._shard_files
        removed = sorted(set(old) - set(now))
        added = sorted(set(now) - set(old))
        changed = sorted(n for n in set(now) & set(old) if now[n] != old[n])
        if not (removed or added or changed):
            return {}
        log.info("shard set changed: added=%s removed=%s changed=%s", added, removed, changed)
        if self.options.role == "coordinator":
            if self.pool is not None:
                await self.pool.remove_shards(removed + changed)
                if self.native_cfg is not None:
                    self.native_cfg.forget(removed + changed)
                self.pool.add_shards(added + changed)
            ctl.set_shard_names(sorted(now))
        else:
            for n in removed + changed:
                await ctl.remove_shard(n)
            o = self.options
            for shard in load_shards(cfg.alias, cfg.shard_config_path, cfg.controller_namespace,
                                     client_factory=self.client_factory,
                                     resync_period=0.0 if o.watch_shards else o.resync_period,
                                     assume_writes=o.assume_writes, sync_binary_data=o.sync_binary_data,
                                     sync_metadata=o.sync_dependent_metadata,
                                     slim=o.slim_shard_cache, start=False, names=set(added + changed)):
                ctl.add_shard(shard)
            self.shards = list(ctl.shards)
        self._shard_files = now
        ctl.enqueue_all()  # fan everything out to new shards; statuses drop removed ones
        return {"added": added, "removed": removed, "changed": changed}

    async def _reload_loop(self, period: float) -> None:
        while True:
            await asyncio.sleep(period)
            self._gauges()
            try:
                await self.reload_shards()
            except Exception as e:  # noqa: BLE001 — a bad kubeconfig must not kill the controller
                log.error("shard reload failed: %s", e)

    def _gauges(self) -> None:
        if self.metrics is None or self.controller is None:
            return
        self.metrics.gauge(C.SHARDS_METRIC, len(self.controller.all_shard_names))
        for shard, n in self.controller.failing_counts().items():
            self.metrics.gauge(C.SHARD_FAILING_METRIC, n, {"shard": shard})
        if self.elector is not None:
            self.metrics.gauge(C.LEADER_METRIC, 1 if self.elector.leading else 0)
        if self.executor_impl:
            self.metrics.gauge(C.EXECUTOR_NATIVE_METRIC, 1 if self.executor_impl == "native" else 0)
        if self.pool is not None:
            for h in self.pool.stats().values():
                for shard, flow in ((h.get("status") or {}).get("flow") or {}).items():
                    for field, name in C.SHARD_CLIENT_METRICS.items():
                        if field in flow:
                            self.metrics.gauge(name, flow[field], {"shard": shard})

    def _ready_checks(self) -> list:
        """`/readyz?verbose`: the caches, and which shard executor implementation runs (and why not the C++ one)."""
        c = self.controller
        out = [("informer-sync", c is not None and c.caches_synced.is_set(), ""),
               ("workers", c is not None and c.ready.is_set(), "")]
        if self.executor_impl:
            out.append(("shard-executors", True, self.executor_impl +
                        (f" (fallback from the C++ executor: {self.executor_fallback})" if self.executor_fallback else "")))
        if self.elector is not None:
            out.append(("leader", True, "leading" if self.elector.leading else "standing by"))
        return out

    def _ready(self) -> bool:
        """Ready once caches synced and workers run — or while standing by for the leader Lease."""
        if self.elector is not None and not self.elector.leading:
            return not self.lost_leadership
        return self.controller is not None and self.controller.ready.is_set() and \
            (self.partitions is None or self.partitions.ready())

    def debug_state(self) -> dict:
        c = self.controller
        out = c.debug_snapshot()
        out["events"] = getattr(self.recorder, "stats", {})
        if self.pool is not None:
            out["executors"] = self.pool.stats()
        if self.partitions is not None:
            out["coordinator_partitions"] = self.partitions.stats()
        if self.relay is not None:
            out["watch_relay"] = dict(self.relay.stats)
        if self.executor_impl:
            out["executor_impl"] = self.executor_impl
            if self.executor_fallback:
                out["executor_fallback"] = self.executor_fallback
        client = self.client
        while client is not None and not hasattr(client, "protocol") and hasattr(client, "inner"):
            client = client.inner  # under a RateLimitedClient
        proto = getattr(client, "protocol", None)
        if proto is not None:  # what the coordinator speaks to the controller apiserver (client-http2)
            out["controller_transport"] = proto
        if self._gc_task is not None:
            out["gc"] = dict(gctune.STATS)
        if self.placement is not None:
            out["cpu_placement"] = {"cpus": self.placement.cpus, "checks": self.placement.checks,
                                    "moves": self.placement.moves}
        if self.elector is not None:
            out["leader"] = {"identity": self.elector.identity, "leading": self.elector.leading,
                             "transitions": self.elector.transitions}
        return out

    async def run(self, stop: asyncio.Event) -> None:
        controller = self.controller or await self.build()
        try:  # `kill -USR1 <pid>` dumps queue/informer state to the log
            asyncio.get_running_loop().add_signal_handler(
                signal.SIGUSR1, lambda: log.warning("debug state: %s", json.dumps(self.debug_state(), default=str)))
        except (NotImplementedError, RuntimeError, ValueError):  # pragma: no cover
            pass
        if self.ops is not None:
            await self.ops.start(self.cfg.health_bind_address or self.cfg.metrics_bind_address)
        if self.gate is None and os.environ.get("NCC_GATED") == "1":
            self.gate = asyncio.Event()  # a child pre-spawned by a warm standby: {"t": "go"} opens it
        if self.cfg.leader_elect and self.options.role != "executor":
            cfg = self.cfg
            self.elector = LeaderElector(self.client, cfg.leader_election_namespace or cfg.controller_namespace,
                                         cfg.leader_election_lease_name, identity_from_env(),
                                         lease_duration=cfg.lease_duration, renew_deadline=cfg.renew_deadline,
                                         retry_period=cfg.retry_period)
            self.gate = asyncio.Event()
        # Everything read-only starts now — informers on every cluster, shard executors (their workers gated
        # while this replica stands by) — so a standby that acquires the Lease only has to open the gates.
        self._start_components(controller)
        run = asyncio.ensure_future(controller.run(stop, gate=self.gate))
        try:
            if self.elector is not None:
                acquire = asyncio.ensure_future(self.elector.acquire(stop))
                done, _ = await asyncio.wait({acquire, run}, return_when=asyncio.FIRST_COMPLETED)
                if acquire not in done or not acquire.result():
                    acquire.cancel()
                    stop.set()
                    await run
                    return
                self.standby_was_warm = controller.caches_synced.is_set() and \
                    (self.pool is None or self.pool.all_synced())

                def lost():
                    self.lost_leadership = True
                    # stop writing before the Lease can expire into another replica's hands: cancel the
                    # workers and kill the executors now instead of letting them drain
                    controller.abort_workers()
                    for group in (self.pool, self.partitions):
                        if group is not None:
                            group.kill()
                    stop.set()
                self._lease_task = asyncio.ensure_future(self.elector.hold(stop, on_lost=lost))
                self.open_gate()
            await run
        finally:
            if not run.done():
                run.cancel()
                await asyncio.gather(run, return_exceptions=True)
            await self.close()

    def _start_components(self, controller: Controller) -> None:
        if self.options.role == "coordinator" and self._relay_ok and self.n_executors > 0:
            from .controller.relay import KINDS, WatchRelay
            infs = {R.TEMPLATES: controller.template_informer, R.WORKGROUPS: controller.workgroup_informer,
                    R.SECRETS: controller.secret_informer, R.CONFIGMAPS: controller.configmap_informer}
            self.relay = WatchRelay([infs[rt] for rt in KINDS], controller.template_informer.store,
                                    self.cfg.controller_namespace)
        for s in self.shards:
            s.start()
        if isinstance(self.recorder, BroadcastRecorder):
            self.recorder.start()
        self.factory.start()
        gated = self.gate is not None and not self.gate.is_set()
        if self.options.role == "coordinator" and self.n_executors > 0:
            env = dict(os.environ)
            env.update(config_to_env(self.cfg))
            env.pop("NCC_COORDINATOR_PART", None)
            env.pop("NCC_GATED", None)
            env.pop("NCC_RELAY", None)
            part, parts = self.coord_part or (0, 1)
            exec_env = dict(env, NCC_RELAY="1") if self.relay is not None else env
            from .controller.native_executor import NativeExecutorConfig, choose
            use_native, why = choose(self.cfg, self.options, self.relay is not None)
            self.executor_impl = "native" if use_native else "python"
            if not use_native:
                # loud: the image requires the C++ executor, so a pod on the Python one is misconfigured or
                # mis-built — a Warning, the executor_native gauge at 0, /readyz?verbose
                self.executor_fallback = why
                if why != "executor-impl: python":
                    log.warning("shard executors: the Python implementation runs instead of the C++ one (%s)", why)
            if self.metrics is not None:
                self.metrics.gauge(C.EXECUTOR_NATIVE_METRIC, 1 if use_native else 0)
            native_cfg = self.native_cfg = NativeExecutorConfig(self.cfg, self.options) if use_native else None
            # One executor group per shard group serves every template key, whatever the number of coordinator
            # partitions: a shard apiserver then serves one executor's watches, not C of them
            # (profiles/r2/c_on_one_shard/: C executors on one shard cost it 12-25 %).
            self.pool = ExecutorPool(controller.all_shard_names, self.n_executors, controller.on_executor_message,
                                     env=exec_env, per_shard=self.per_shard, gated=gated, relay=self.relay,
                                     native_config=native_cfg, on_stream=controller.on_executor_stream)
            if native_cfg is not None:
                self._cred_task = asyncio.ensure_future(native_cfg.refresh_loop(self.pool))
            self.pool.start()
            if parts > 1 and part == 0:
                # the children own keys ≡ p mod C: their executor reports are forwarded raw by the report table,
                # and a child that comes up (or back) gets every executor to pass over its keys again
                pool = self.pool
                self.partitions = CoordinatorPartitions(
                    parts, env, gated=gated, on_child_ready=lambda p: pool.resync_partition(p, parts))
                controller.reports.set_partition(0, parts)
                controller.forward_reports = self.partitions.forward
                self.partitions.start()
            recheck = float(os.environ.get("NCC_CPU_AFFINITY_RECHECK_S", "30"))
            if self.placement is not None and recheck > 0:
                self._placement_task = asyncio.ensure_future(self.placement.loop(
                    recheck, self._child_pids, controller.queue.idle))
        if self.cfg.mode == "native":
            gctune.tune()  # thresholds and a freeze only: the start-up garbage was collected in build()
            # NCC_GC_FREEZE="<period>,<generation collected first, or none>" (experiments; default "1,none":
            # freeze every second, after a generation-0 pass when no automatic one ran since the last freeze);
            # NCC_GC_FULL_S: unfreeze + full collection this often, at an idle moment when there is one
            period, _, gen = os.environ.get("NCC_GC_FREEZE", "1,none").partition(",")
            queue = self.controller.queue
            self._gc_task = asyncio.ensure_future(gctune.freeze_loop(
                float(period), collect=None if gen in ("", "none", "blind") else int(gen),
                full_period=float(os.environ.get("NCC_GC_FULL_S", "300")), idle=queue.idle,
                young=gen != "blind"))
        self._lag_task = loopmon.start(self.options.role)
        if self.cfg.mode == "native" and self.options.role != "executor" and self.cfg.shard_reload_period > 0:
            self._reload_task = asyncio.ensure_future(self._reload_loop(self.cfg.shard_reload_period))
        topo_file = os.environ.get("NCC_TOPOLOGY_FILE")
        if topo_file and self.options.role == "coordinator" and not os.environ.get("NCC_COORDINATOR_PART"):
            with open(topo_file + ".tmp", "w") as f:  # for benchmarks / operators: what auto-sizing picked
                json.dump(self.topology(), f)
            os.replace(topo_file + ".tmp", topo_file)
        log.info("nexus-configuration-controller %s starting: mode=%s role=%s alias=%s namespace=%s shards=%s "
                 "executors=%d×%d (%s) workers=%d%s", __version__, self.cfg.mode, self.options.role, self.cfg.alias,
                 self.cfg.controller_namespace, controller.all_shard_names, self.n_executors, self.per_shard,
                 self.executor_impl or "in-process", self.options.workers, " (standing by)" if gated else "")

    def _child_pids(self) -> list[int]:
        return [h.proc.pid for group in (self.pool, self.partitions) if group is not None
                for h in group.handles if h.proc is not None and h.proc.returncode is None]

    def _shard_owner_filter(self, infs: dict):
        """A partitioned executor's filter for shard Secrets/ConfigMaps: owned by one of its partition's
        templates, unowned, or referenced by one of them — a copy another partition's template owns is still
        one this partition writes to (with server-side apply it must see the other owners' refs, which an
        apply without them would drop)."""
        o = self.options
        if o.partition is None:
            return None
        tstore = infs[R.TEMPLATES].store

        def referenced(ns: str, name: str) -> bool:
            key = f"{ns}/{name}"
            return bool(tstore.by_index("secret", key) or tstore.by_index("configmap", key))
        return partition_owner_filter(*o.partition, referenced=referenced)

    def topology(self) -> dict:
        """The process layout this coordinator chose (automatic sizing or overrides)."""
        parts = self.coord_part[1] if self.coord_part else 1
        return {"shard_groups": self.n_executors, "executors_per_shard": self.per_shard,
                "coordinator_partitions": parts, "executor_impl": self.executor_impl or "in-process",
                "executor_processes": len(self.pool.handles) if self.pool is not None else 0,
                "watch_relay": self.relay is not None, "cpu_affinity": self.cpu_affinity or "none"}

    def open_gate(self) -> None:
        """Leading now (or released by the parent): start reconciling here and in every child process."""
        if self.gate is None or self.gate.is_set():
            return
        log.info("gate open: starting workers (role=%s)", self.options.role)
        for group in (self.pool, self.partitions):
            if group is not None:
                group.open_gate()
        self.gate.set()

    async def close(self) -> None:
        log.info("closing (role=%s)", self.options.role)
        for t in (self._lease_task, self._reload_task, self._gc_task, self._cred_task, self._lag_task,
                  self._placement_task):
            if t is not None:
                t.cancel()
                await asyncio.gather(t, return_exceptions=True)
        if self.partitions is not None:
            await self.partitions.stop()
        if self.pool is not None:
            await self.pool.stop()
        if self.relay is not None:
            self.relay.dump_trace()
        if isinstance(self.recorder, BroadcastRecorder):
            await self.recorder.stop()
        await self.factory.stop()
        log.debug("controller informers stopped")
        for s in self.shards:
            await s.stop()
        log.debug("shards stopped")
        if self.elector is not None and self.elector.leading:
            await self.elector.release()
        await self.client.close()
        if self.ops is not None:
            await self.ops.stop()
        if self.metrics is not None:
            self.metrics.close()
        log.info("closed (role=%s)", self.options.role)
        if os.environ.get("NCC_CPU_REPORT"):
            import resource
            ru = resource.getrusage(resource.RUSAGE_SELF)
            infs = [self.factory] + [s.factory for s in self.shards]
            counts = {i.name: (i.events, getattr(i, "echoes", 0), i.filtered) for f in infs for i in f.informers()}
            log.warning("informer events/echoes/filtered: %s", counts)
            log.warning("cpu report role=%s user_s=%.3f sys_s=%.3f stats=%s events=%s gc=%s", self.options.role,
                        ru.ru_utime, ru.ru_stime, self.controller.stats, getattr(self.recorder, "stats", {}),
                        gctune.STATS)


def setup_signal_handler(stop: asyncio.Event) -> None:
    """signals.SetupSignalHandler: first SIGINT/SIGTERM cancels, a second one exits immediately."""
    loop = asyncio.get_running_loop()
    hits = {"n": 0}

    def on_signal():
        hits["n"] += 1
        if hits["n"] > 1:
            os._exit(1)
        stop.set()

    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, on_signal)
        except (NotImplementedError, RuntimeError):  # pragma: no cover - non-main thread
            pass


async def _amain(cfg: AppConfig, control_fd: int | None = None) -> int:
    stop = asyncio.Event()
    setup_signal_handler(stop)
    app = App(cfg)
    try:
        await app.build()
    except Exception as e:  # noqa: BLE001
        log.error("Error building controller: %s", e)
        return 1
    watcher = None
    if control_fd is not None:
        # a coordinator partition started by its parent: report readiness; the parent closing the channel
        # (or dying) ends this process
        import socket

        from .controller.ipc import Channel
        reader, writer = await asyncio.open_connection(sock=socket.socket(fileno=control_fd))
        channel = Channel(reader, writer)
        app.controller.on_ready = lambda: channel.send({"t": "ready"})
        ctl = app.controller

        def fold(buf, start):  # executor reports on this partition's keys, forwarded raw by the parent
            return ctl.on_executor_stream(-1, buf, start)

        async def watch_parent():
            while True:
                batch = await channel.recv_folded(fold)
                if batch is None:
                    break
                if any(isinstance(m, dict) and m.get("t") == "go" for m in batch):
                    app.open_gate()  # the parent acquired the Lease
            stop.set()
        watcher = asyncio.ensure_future(watch_parent())
    try:
        await app.run(stop)
    finally:
        if watcher is not None:
            watcher.cancel()
    return 1 if app.lost_leadership else 0


# klog.InitFlags(nil) + flag.Parse() (main.go:36-37): the reference binary accepts klog's flags.  `-v N`
# maps onto the log level (the reference logs reconcile detail at V(4)); the output-routing flags are
# accepted and ignored, since logs always go to stdout as structured lines here.
_KLOG_VALUE_FLAGS = ("log_dir", "log_file", "log_file_max_size", "stderrthreshold", "vmodule", "log_backtrace_at")
_KLOG_BOOL_FLAGS = ("logtostderr", "alsologtostderr", "add_dir_header", "skip_headers", "skip_log_headers",
                    "one_output")


def _go_style_flags(argv: list) -> list:
    """Go's flag package takes `-name`, `--name`, `-name=value`; argparse wants `--name` for long names."""
    out = []
    for a in argv:
        if a.startswith("-") and not a.startswith("--") and len(a.split("=", 1)[0]) > 2:
            a = "-" + a
        out.append(a)
    return out


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="python -m ncc", description="Nexus multi-cluster configuration controller")
    p.add_argument("--config-dir", default=None, help="directory holding appconfig.yaml (default: cwd)")
    p.add_argument("--version", action="store_true")
    p.add_argument("--check-shards", action="store_true",
                   help="preflight: list every kind on the controller cluster and each shard, print one JSON line "
                        "per cluster and exit (0: all answered)")
    p.add_argument("--control-fd", type=int, default=None, help=argparse.SUPPRESS)  # coordinator partitions
    p.add_argument("-v", "--v", type=int, default=None, metavar="N",
                   help="klog verbosity: N>=4 logs at DEBUG (overrides log-level), N<4 leaves log-level as set")
    for f in _KLOG_VALUE_FLAGS:
        p.add_argument(f"--{f}", default=None, help=argparse.SUPPRESS)
    for f in _KLOG_BOOL_FLAGS:
        p.add_argument(f"--{f}", nargs="?", const="true", default=None, help=argparse.SUPPRESS)
    args = p.parse_args(_go_style_flags(list(sys.argv[1:] if argv is None else argv)))
    from .proclimits import raise_nofile_limit
    raise_nofile_limit()
    if args.version:
        print(__version__)
        return 0
    try:
        cfg = load_config(args.config_dir)
    except (ValueError, OSError) as e:
        print(f"configuration error: {e}", file=sys.stderr)
        return 1
    except Exception as e:  # noqa: BLE001 - a malformed appconfig.yaml (yaml.YAMLError)
        print(f"configuration error: {type(e).__name__}: {e}", file=sys.stderr)
        return 1
    if args.v is not None and args.v >= 4:
        cfg.log_level = "DEBUG"
    configure_logging(cfg.log_level, cfg.log_format)
    if args.check_shards:
        from .preflight import run as preflight
        return preflight(cfg)
    from . import sampler
    sampler.start("coordinator" + os.environ.get("NCC_COORDINATOR_PART", "").replace("/", "of"))
    prof_path = os.environ.get("NCC_PROFILE")
    if prof_path:  # host-side profiling of the control loop: NCC_PROFILE=/path/out.prof
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
        part = os.environ.get("NCC_COORDINATOR_PART", "").replace("/", "of")
        try:
            return asyncio.run(_amain(cfg, args.control_fd))
        finally:
            prof.disable()
            prof.dump_stats(prof_path + (f".coordinator{part}" if part else ""))
    return asyncio.run(_amain(cfg, args.control_fd))
