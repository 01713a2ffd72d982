#!/usr/bin/env python
"""Headline benchmark: objects synced/s and p50/p99 controller→shard propagation latency at N shards.

Metric and topology come from BASELINE.json ("objects synced/sec + p50 controller->shard latency
at 1/2/4/8 shards").  `--gpus N` is the number of shard clusters: under
`torch.distributed.run --nproc-per-node N` every rank hosts one shard kube-apiserver process (the
shard clusters are 8×MI355X nodes; one rank per GPU == one shard per GPU), rank 0 additionally
hosts the controller-cluster apiserver and runs the controller (`python -m ncc`) as a separate
process exactly as deployed.  Ranks rendezvous over gloo (no tensors are exchanged; RCCL is not
involved in a control plane).

Workload (synthetic, BASELINE.json config 3 shape by default): T NexusAlgorithmTemplates, each
referencing 1 Secret + 1 ConfigMap, in namespace `nexus`.  Warm-up = cold start (controller
boots against pre-seeded objects and fans everything out) + W update waves; then K timed waves.
A wave bumps every template's `versionTag` and every Secret/ConfigMap payload in one burst on
the controller cluster (the wave's request is sent and decoded by the controller apiserver before the
clock starts; a timed step commits it); the step ends when every shard has committed all 3·T new versions.
Per-object latency = shard commit time − controller commit time (server-side clocks, same host).

value = K · 3 · T · N / (wall time of the K timed waves, max over ranks)   [objects/s, weak scaling]
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import json
import os
import shutil
import signal
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "objects synced/sec + p50 controller->shard latency at 1/2/4/8 shards"
NS = "nexus"
# bench mode -> controller environment
MODES = {"native": {"NEXUS__MODE": "native"},
         "compat": {"NEXUS__MODE": "compat"},
         "compat-unthrottled": {"NEXUS__MODE": "compat", "NEXUS__CLIENT_QPS": "-1"}}
MARKERS = ["nexusalgorithmtemplates=spec.container.versionTag", "secrets=data.version", "configmaps=data.version"]


def parse_args(argv=None):
    p = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")),
                   help="number of shard clusters (one per rank/GPU)")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--templates", type=int, default=1000)
    p.add_argument("--payload", type=int, default=512, help="bytes per Secret/ConfigMap payload")
    p.add_argument("--mode", default="native", choices=list(MODES),
                   help="native | compat (reference semantics incl. client-go's 5 QPS/10 burst) | "
                        "compat-unthrottled (reference semantics without the client-side limiter)")
    p.add_argument("--workers", type=int, default=0, help="controller workers (0 = mode default)")
    p.add_argument("--timeout", type=float, default=600.0, help="per-wave convergence timeout (s)")
    p.add_argument("--keep", action="store_true", help="keep the work directory")
    p.add_argument("--pin", choices=("none", "l3", "controller"), default="none",
                   help="l3: the controller (coordinator + executors) on the least busy L3 domain of the CPUs this job "
                        "may use, the fake apiservers on the next one; controller: only the controller pinned (one "
                        "rank only; experiments)")
    p.add_argument("--extra-env", action="append", default=[], help="KEY=VAL passed to the controller process")
    p.add_argument("--shard-latency-ms", type=float, default=0.0,
                   help="added to every request a shard apiserver serves (emulates controller->shard RTT)")
    p.add_argument("--shard-jitter-ms", type=float, default=0.0,
                   help="uniform extra delay 0..J ms per shard request, on top of --shard-latency-ms")
    p.add_argument("--no-tls-run", action="store_true",
                   help="skip the second, production-transport run (TLS everywhere, product defaults) whose results "
                        "go into the JSON line as tls_* keys")
    p.add_argument("--product-defaults", action="store_true",
                   help="run the controller with the product's defaults (cpu-affinity none, client-http2 auto) "
                        "instead of the bench's (l3, on)")
    p.add_argument("--tls", action="store_true",
                   help="every apiserver serves HTTPS with x509 client auth (throwaway CA), as kind/EKS clusters do")
    p.add_argument("--shards-per-rank", type=int, default=1,
                   help="experiments only: shard apiservers hosted per rank (the driver contract is 1)")
    p.add_argument("--stages", action="store_true",
                   help="trace where each object's latency goes (controller commit -> coordinator relay -> "
                        "executor receive -> executor dequeue -> shard commit) and report p50/p99 per stage")
    return p.parse_args(argv)


# ------------------------------------------------------------------ distributed plumbing
class Dist:
    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist
        self._cuda = None

    def all_gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def broadcast(self, obj):
        if self.dist is None:
            return obj
        box = [obj]
        self.dist.broadcast_object_list(box, src=0)
        return box[0]

    def sync(self):
        """barrier + torch.cuda.synchronize() (the bench contract); GPUs do no work in a control plane."""
        if self.dist is not None:
            self.dist.barrier()
        if self._cuda is None:
            try:
                import torch
                self._cuda = torch.cuda.is_available()
                if self._cuda:
                    torch.cuda.set_device(self.local_rank % max(torch.cuda.device_count(), 1))
            except Exception:  # noqa: BLE001
                self._cuda = False
        if self._cuda:
            import torch
            torch.cuda.synchronize()

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        return max(self.all_gather(x))

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def _shard_transport(ctl_debug) -> str:
    flows = ((ctl_debug or {}).get("executor_flow") or {}).values()
    h2 = [f.get("http2") for f in flows if isinstance(f, dict)]
    if not h2:
        return "n/a"
    return "http2" if all(h2) else ("http/1.1" if not any(h2) else "mixed")


# ------------------------------------------------------------------ workload
def wave_objects(T: int, version: int, payload: int) -> list:
    """One wave: per template its Secret, its ConfigMap, then the template itself (dependencies first,
    as a user rolling out a new config version would)."""
    from ncc.testing.workload import configmap_name, make_configmap, make_secret, make_template, secret_name
    items = []
    for i in range(T):
        items.append(make_secret(secret_name(i), NS, payload=payload, version=version))
        items.append(make_configmap(configmap_name(i), NS, payload=payload, version=version))
        items.append(make_template(i, NS, secrets=[secret_name(i)], configmaps=[configmap_name(i)],
                                   version=f"v{version}"))
    return items


def wave_body(T: int, version: int, payload: int, stage_id=None) -> bytes:
    """/_fake/apply (or, with `stage_id`, /_fake/stage) request body, generated before the timed region:
    the load generator's own work is not part of the system under test.  The server commits in slices
    of 100 objects and lets watches flush in between, like a real apiserver under many concurrent writers."""
    body = {"items": wave_objects(T, version, payload), "yield_every": 100}
    if stage_id is not None:
        body["id"] = stage_id
    return json.dumps(body).encode()


def want(T: int, version: int) -> list:
    return [{"plural": "nexusalgorithmtemplates", "value": f"v{version}", "count": T},
            {"plural": "secrets", "value": base64.b64encode(str(version).encode()).decode(), "count": T},
            {"plural": "configmaps", "value": str(version), "count": T}]


async def set_shard_latency(urls: list, latency_ms: float, jitter_ms: float, ssl_ctx=None) -> None:
    """Drive the fake apiservers' fault hook (ncc/fakeapi/server.py `Faults`): every API request a shard
    serves is delayed by latency + U(0, jitter) ms before it is processed, so each controller->shard write
    pays a network round trip as it would against a remote cluster."""
    import aiohttp
    async with aiohttp.ClientSession(connector=aiohttp.TCPConnector(ssl=ssl_ctx) if ssl_ctx else None) as session:
        for u in urls:
            await post(session, f"{u}/_fake/faults", {"latency_ms": latency_ms, "jitter_ms": jitter_ms})


def client_ssl(pki):
    """The load generator's own client context for the HTTPS apiservers (their CA, the client certificate)."""
    import ssl
    ctx = ssl.create_default_context(cafile=pki.ca_cert)
    ctx.load_cert_chain(pki.client_cert, pki.client_key)
    return ctx


async def post(session, url, body, timeout=None):
    import aiohttp
    data = body if isinstance(body, bytes) else json.dumps(body)
    async with session.post(url, data=data, headers={"Content-Type": "application/json"},
                            timeout=aiohttp.ClientTimeout(total=timeout)) as r:
        r.raise_for_status()
        return await r.json()


def cpu_seconds(named: dict, rss: dict | None = None, sys_out: dict | None = None) -> dict:
    """user+sys CPU seconds per named process; `coordinator` also reports its executor children.
    With `rss` given, resident memory (MiB) per process is recorded there too; with `sys_out`, the
    kernel-mode part of the CPU seconds."""
    import psutil
    out = {}
    sys_out = {} if sys_out is None else sys_out
    for name, proc in named.items():
        if proc is None:
            continue
        try:
            p = psutil.Process(proc.pid)
            t = p.cpu_times()
            out[name] = t.user + t.system
            sys_out[name] = t.system
            if rss is not None:
                rss[name] = round(p.memory_info().rss / 2**20, 1)
            if name == "coordinator":
                # children: shard executors (ncc-executor / -m ncc.executor) and, on large hosts, the
                # coordinator partitions (-m ncc), whose cost is the coordinator's
                ex, co = [], []
                for c in p.children(recursive=True):
                    try:
                        cmd = " ".join(c.cmdline())
                    except (psutil.Error, OSError):
                        continue
                    (ex if ("ncc-executor" in cmd or "ncc.executor" in cmd) else co).append(c)
                ext = [c.cpu_times() for c in ex]
                cot = [c.cpu_times() for c in co]
                out["executors"] = sum(t.user + t.system for t in ext)
                sys_out["executors"] = sum(t.system for t in ext)
                if cot:  # partitioned: the parent alone too (it relays and routes every key's reports)
                    out["coordinator-parent"] = out[name]
                out[name] += sum(t.user + t.system for t in cot)
                sys_out[name] += sum(t.system for t in cot)
                if rss is not None:
                    rss["executors"] = round(sum(c.memory_info().rss for c in ex) / 2**20, 1)
                    rss[name] += round(sum(c.memory_info().rss for c in co) / 2**20, 1)
        except (psutil.Error, OSError):
            pass
    return out


# ------------------------------------------------------------------ host (box speed vs code speed)
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def cgroup_cpu() -> dict:
    """The job's CPU quota and its throttling counters (cgroup v2 `cpu.max` / `cpu.stat`, or v1 equivalents)."""
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
            out["quota_cpus"] = None if q == "max" else round(int(q) / int(p), 2)
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for ln in f:
                k, v = ln.split()
                if k in ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec"):
                    out[k] = int(v)
    except (OSError, ValueError):
        try:  # cgroup v1
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = int(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                p = int(f.read())
            out["quota_cpus"] = None if q < 0 else round(q / p, 2)
            with open("/sys/fs/cgroup/cpu/cpu.stat") as f:
                for ln in f:
                    k, v = ln.split()
                    if k == "throttled_time":
                        out["throttled_usec"] = int(v) // 1000
                    elif k in ("nr_periods", "nr_throttled"):
                        out[k] = int(v)
        except (OSError, ValueError):
            pass
    return out


def calibrate() -> dict:
    """Fixed work timed on this box: a pure-Python loop (dict/str work like the coordinator's) and the C++
    executor's own `--calibrate` (relayed-line scan, fingerprint, render, crc32).  A slow box shows here
    before it shows in objects/s."""
    def py_loop():
        d = {}
        for i in range(200_000):
            k = "nexus/algo-%05d" % (i % 1000)
            d[k] = d.get(k, 0) + len(k)
        return d
    best = 1e9
    for _ in range(5):
        t0 = time.perf_counter()
        py_loop()
        best = min(best, time.perf_counter() - t0)
    out = {"python_loop_ms": round(best * 1000, 2)}
    exe = os.path.join(ROOT, "ncc", "bin", "ncc-executor")
    if os.path.exists(exe):
        try:
            r = subprocess.run([exe, "--calibrate"], capture_output=True, text=True, timeout=60)
            c = json.loads(r.stdout.strip().splitlines()[-1])
            out.update({f"cpp_{k}": v for k, v in c.items() if k.endswith("_ns")})
        except (OSError, ValueError, IndexError, subprocess.TimeoutExpired):
            pass
    return out


def ctx_switches(named: dict) -> dict:
    """Voluntary / involuntary context switches per named process (executors summed under the coordinator)."""
    import psutil
    out = {}
    for name, proc in named.items():
        if proc is None:
            continue
        try:
            p = psutil.Process(proc.pid)
            c = p.num_ctx_switches()
            out[name] = [c.voluntary, c.involuntary]
            if name == "coordinator":
                ex = [0, 0]
                for k in p.children(recursive=True):
                    try:
                        if "ncc-executor" in " ".join(k.cmdline()) or "ncc.executor" in " ".join(k.cmdline()):
                            kc = k.num_ctx_switches()
                            ex[0] += kc.voluntary
                            ex[1] += kc.involuntary
                    except (psutil.Error, OSError):
                        pass
                out["executors"] = ex
        except (psutil.Error, OSError):
            pass
    return out


def host_busy() -> tuple[float, float] | None:
    """(busy, total) CPU-seconds of the whole host so far (/proc/stat, not namespaced): the delta over the
    timed waves, minus this job's own CPU, is what other tenants ran on the machine meanwhile."""
    try:
        with open("/proc/stat") as f:
            v = [int(x) for x in f.readline().split()[1:]]
    except (OSError, ValueError):
        return None
    hz = os.sysconf("SC_CLK_TCK")
    idle = v[3] + (v[4] if len(v) > 4 else 0)
    return (sum(v) - idle) / hz, sum(v) / hz


def l3_pin_sets(k: int = 2) -> list[list[int]] | None:
    """The CPUs of the `k` least busy L3 domains this process may run on (busy: /proc/stat over 0.3 s)."""
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except OSError:
        return None
    doms: dict[int, list[int]] = {}
    for c in allowed:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list") as f:
                dom = min(_cpu_list(f.read()))
        except (OSError, ValueError):
            return None
        doms.setdefault(dom, []).append(c)
    if len(doms) < k:
        return None

    def per_cpu():
        out = {}
        with open("/proc/stat") as f:
            for ln in f:
                if ln.startswith("cpu") and ln[3:4].isdigit():
                    parts = ln.split()
                    v = [int(x) for x in parts[1:]]
                    out[int(parts[0][3:])] = (sum(v) - v[3] - (v[4] if len(v) > 4 else 0), sum(v))
        return out
    a = per_cpu()
    time.sleep(0.3)
    b = per_cpu()

    def busy(cpus):
        db = sum(b[c][0] - a[c][0] for c in cpus if c in a and c in b)
        dt = sum(b[c][1] - a[c][1] for c in cpus if c in a and c in b)
        return db / dt if dt else 1.0
    ranked = sorted(doms.values(), key=busy)
    return ranked[:k]


def _cpu_list(text: str) -> list[int]:
    out = []
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


class Placement:
    """Where the busy processes ran during the timed waves: every 20 ms, the CPU each was last on
    (/proc/<pid>/stat), mapped to its physical core (SMT siblings) and L3 domain.  Two of them on one
    physical core at once halve each other's speed — a run-to-run variance the calibration loop, timed alone,
    does not see.  Reported: the share of samples in which a process shared its core with another one, the
    distinct cores and L3 domains used, and the CPUs the job may run on."""

    def __init__(self, named: dict):
        import threading
        self.named = named
        self.samples = 0
        self.shared: dict[str, int] = {}
        self.cores: dict[str, set] = {}
        self.l3: set = set()
        self._stop = threading.Event()
        self._core: dict[int, int] = {}
        self._l3: dict[int, int] = {}
        self._t = threading.Thread(target=self._run, daemon=True)

    def _topo(self, cpu: int) -> tuple[int, int]:
        c = self._core.get(cpu)
        if c is None:
            base = f"/sys/devices/system/cpu/cpu{cpu}"
            try:
                with open(f"{base}/topology/thread_siblings_list") as f:
                    c = min(_cpu_list(f.read()))
            except (OSError, ValueError):
                c = cpu
            try:
                with open(f"{base}/cache/index3/shared_cpu_list") as f:
                    self._l3[cpu] = min(_cpu_list(f.read()))
            except (OSError, ValueError):
                self._l3[cpu] = -1
            self._core[cpu] = c
        return c, self._l3[cpu]

    def _pids(self) -> dict:
        import psutil
        out = {}
        for name, proc in self.named.items():
            if proc is None:
                continue
            out[name] = proc.pid
            if name == "coordinator":
                try:
                    for i, c in enumerate(psutil.Process(proc.pid).children(recursive=True)):
                        out[f"coordinator-child{i}"] = c.pid
                except (psutil.Error, OSError):
                    pass
        return out

    def _run(self) -> None:
        pids = self._pids()
        while not self._stop.wait(0.02):
            where = {}
            for name, pid in pids.items():
                try:
                    with open(f"/proc/{pid}/stat") as f:
                        fields = f.read().rsplit(")", 1)[1].split()
                    if fields[0] not in ("R",):
                        continue  # only processes running (or runnable) right now compete for a core
                    cpu = int(fields[36])
                except (OSError, IndexError, ValueError):
                    continue
                where[name] = self._topo(cpu)
            self.samples += 1
            by_core: dict[int, int] = {}
            for core, l3 in where.values():
                by_core[core] = by_core.get(core, 0) + 1
                self.l3.add(l3)
            for name, (core, _) in where.items():
                self.cores.setdefault(name, set()).add(core)
                if by_core[core] > 1:
                    self.shared[name] = self.shared.get(name, 0) + 1

    def start(self) -> "Placement":
        self._t.start()
        return self

    def stop(self) -> dict:
        self._stop.set()
        self._t.join(timeout=2)
        try:
            allowed = len(os.sched_getaffinity(0))
        except OSError:
            allowed = None
        n = max(1, self.samples)
        return {"samples": self.samples, "allowed_cpus": allowed, "l3_domains_used": len(self.l3),
                "core_shared_share": {k: round(v / n, 3) for k, v in sorted(self.shared.items())},
                "cores_used": {k: len(v) for k, v in sorted(self.cores.items())}}


def child_pids(proc) -> set:
    """PIDs of every process under the controller (coordinator partitions, executors)."""
    import psutil
    try:
        return {c.pid for c in psutil.Process(proc.pid).children(recursive=True)}
    except (psutil.Error, OSError):
        return set()


def pct(xs, q):
    if not xs:
        return None
    xs = sorted(xs)
    k = min(len(xs) - 1, max(0, int(round(q / 100.0 * (len(xs) - 1)))))
    return xs[k]


# ------------------------------------------------------------------ latency stages (--stages)
KIND_INDEX = {"nexusalgorithmtemplates": 0, "secrets": 2, "configmaps": 3}
STAGES = ("relay", "ipc", "queue", "write")


def _first_at_or_after(ts: list, t: int):
    import bisect
    i = bisect.bisect_left(ts, t)
    return ts[i] if i < len(ts) else None


def stage_breakdown(trace_dir: str, ctrl_times: list, shard_waves: list, executor: int = 0) -> dict | None:
    """Per object of the timed waves on shard 0: controller commit -> coordinator relay (`relay`) -> executor
    receive (`ipc`) -> executor worker dequeue of the owning template key (`queue`: coalescing and work-queue
    wait) -> shard commit (`write`: the pass up to the shard apiserver committing the object).  p50/p99 per
    stage, and the mean stage split of the slowest 1 % of objects (who owns the p99)."""
    import glob as _glob
    relay: dict = {}
    recv: dict = {}
    deq: dict = {}
    for f in _glob.glob(os.path.join(trace_dir, "relay-*.tsv")):
        with open(f) as fh:
            for ln in fh:
                k, key, t = ln.rstrip("\n").split("\t")
                relay.setdefault((int(k), key), []).append(int(t))
    ex_files = sorted(_glob.glob(os.path.join(trace_dir, f"executor-{executor}-*.tsv")))
    if not relay or not ex_files:
        return None
    for f in ex_files:
        with open(f) as fh:
            for ln in fh:
                w, k, key, t = ln.rstrip("\n").split("\t")
                if w == "r":
                    recv.setdefault((int(k), key), []).append(int(t))
                else:
                    deq.setdefault(key, []).append(int(t))
    for dct in (relay, recv, deq):
        for v in dct.values():
            v.sort()
    rows = []
    for ctrl, wave in zip(ctrl_times, shard_waves):
        for marker, objs in wave.items():
            plural = marker.split("=", 1)[0]
            kind = KIND_INDEX.get(plural)
            if kind is None:
                continue
            c = ctrl[marker]
            for k, t_s in objs.items():
                key = k.split(":", 1)[-1]
                t_c = c.get(key)
                if t_c is None:
                    continue
                t_r = _first_at_or_after(relay.get((kind, key), []), t_c)
                t_e = _first_at_or_after(recv.get((kind, key), []), t_r if t_r is not None else t_c)
                name = key.split("/", 1)[-1]
                owner = name if kind == 0 else name.rsplit("-", 1)[0]  # workload: <template>-secret/-config
                t_q = _first_at_or_after(deq.get(f"template/{key.split('/', 1)[0]}/{owner}", []),
                                         t_e if t_e is not None else t_c)
                if None in (t_r, t_e, t_q) or not (t_c <= t_r <= t_e <= t_q <= t_s):
                    continue
                rows.append((t_s - t_c, t_r - t_c, t_e - t_r, t_q - t_e, t_s - t_q, plural))
    if not rows:
        return None
    out = {"objects": len(rows)}
    for i, name in enumerate(("total",) + STAGES):
        xs = [r[i] / 1e6 for r in rows]
        out[name] = {"p50_ms": round(pct(xs, 50), 2), "p99_ms": round(pct(xs, 99), 2)}
    by_kind = {}
    for r in rows:
        by_kind.setdefault(r[5], []).append(r[0] / 1e6)
    out["total_by_kind"] = {k: {"p50_ms": round(pct(v, 50), 2), "p99_ms": round(pct(v, 99), 2)}
                            for k, v in sorted(by_kind.items())}
    rows.sort(key=lambda r: r[0])
    tail = rows[-max(1, len(rows) // 100):]
    out["p99_tail_mean_ms"] = {name: round(sum(r[i + 1] for r in tail) / len(tail) / 1e6, 2)
                               for i, name in enumerate(STAGES)}
    out["p99_owner"] = max(out["p99_tail_mean_ms"], key=out["p99_tail_mean_ms"].get)
    return out


# ------------------------------------------------------------------ main
async def run(args, d: Dist) -> dict | None:
    import aiohttp
    from ncc.kube.kubeconfig import render_kubeconfig
    from ncc.testing.env import spawn_fakeapi, wait_port_file

    work = tempfile.mkdtemp(prefix=f"ncc-bench-r{d.rank}-")
    procs = []
    pki = ssl_ctx = None
    try:
        if args.tls:  # one CA for the job (all ranks are on one node): rank 0 makes it, the others read it
            from ncc.testing.pki import PKI, make_pki
            pdir = None
            if d.rank == 0:
                pdir = make_pki(os.path.join(work, "pki")).dir
            pdir = d.broadcast(pdir)
            j_ = lambda n: os.path.join(pdir, n)  # noqa: E731
            pki = PKI(pdir, j_("ca.crt"), j_("server.crt"), j_("server.key"), j_("client.crt"), j_("client.key"))
            ssl_ctx = client_ssl(pki)
        extra = sum((["--marker", m] for m in MARKERS), [])
        S = max(1, args.shards_per_rank)
        pin_sets = l3_pin_sets(2) if args.pin != "none" and d.world == 1 else None

        def pin(proc, which: int) -> None:
            if pin_sets and (which == 0 or args.pin == "l3"):
                try:
                    os.sched_setaffinity(proc.pid, pin_sets[which])
                except OSError:
                    pass
        my_urls = []
        for j in range(S):
            pf = os.path.join(work, f"shard{j}.url")
            procs.append(spawn_fakeapi(f"shard-{d.rank * S + j}", pf, extra=extra, pki=pki))
            pin(procs[-1], 1)
            my_urls.append(wait_port_file(pf, procs[-1]))
        my_url = my_urls[0]
        if args.shard_latency_ms or args.shard_jitter_ms:
            await set_shard_latency(my_urls, args.shard_latency_ms, args.shard_jitter_ms, ssl_ctx)
        urls = [u for us in d.all_gather(my_urls) for u in us]
        ctrl_url = None
        controller = None
        T = args.templates
        if d.rank == 0:
            cpf = os.path.join(work, "controller.url")
            procs.append(spawn_fakeapi("controller", cpf, extra=extra, pki=pki))
            pin(procs[-1], 1)
            ctrl_url = wait_port_file(cpf, procs[-1])
            ctrl_proc = procs[-1]
            shard_dir = os.path.join(work, "shards")
            os.makedirs(shard_dir)
            tls = dict(ca_data=pki.ca_data, client_cert_data=pki.client_cert_data,
                       client_key_data=pki.client_key_data) if pki is not None else {}
            for i, u in enumerate(urls):
                with open(os.path.join(shard_dir, f"shard-{i}.kubeconfig"), "w") as f:
                    f.write(render_kubeconfig(u, f"shard-{i}", **tls))
            ckc = os.path.join(work, "controller.kubeconfig")
            with open(ckc, "w") as f:
                f.write(render_kubeconfig(ctrl_url, "controller", **tls))
        connector = aiohttp.TCPConnector(ssl=ssl_ctx) if ssl_ctx is not None else None
        async with aiohttp.ClientSession(connector=connector) as session:
            if d.rank == 0:
                await post(session, f"{ctrl_url}/_fake/apply", {"items": wave_objects(T, 0, args.payload)})
                env = dict(os.environ)
                env.update({"NEXUS__CONTROLLER_CONFIG_PATH": ckc, "NEXUS__SHARD_CONFIG_PATH": shard_dir,
                            "NEXUS__CONTROLLER_NAMESPACE": NS, "NEXUS__ALIAS": "controller-cluster",
                            "NEXUS__LOG_LEVEL": "WARNING",
                            "PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", "")})
                env.update(MODES[args.mode])
                if args.workers:  # native: per-process workers (otherwise the config's native-workers default)
                    env["NEXUS__WORKERS"] = str(args.workers)
                    env["NEXUS__NATIVE_WORKERS"] = str(args.workers)
                for kv in args.extra_env:
                    k, _, v = kv.partition("=")
                    env[k] = v
                env["NCC_TOPOLOGY_FILE"] = os.path.join(work, "topology.json")
                # the deployment knob (Helm controller.cpuAffinity, off by default) set to l3: the bench hosts are
                # shared multi-CCD machines, where the coordinator and its executors on one L3 domain run in the
                # fast regime (ncc/affinity.py); reported as controller_sizing.cpu_affinity
                if not args.product_defaults:
                    env.setdefault("NCC_CPU_AFFINITY", "l3")
                # the executors speak HTTP/2 to the shard apiservers, as client-go does to a kube-apiserver (by
                # ALPN on TLS; here, on the bench's cleartext connections, with prior knowledge): `--extra-env
                # NEXUS__CLIENT_HTTP2=off` measures the HTTP/1.1 pool instead (BENCHMARKS.md "HTTP/2")
                if not args.product_defaults:
                    env.setdefault("NEXUS__CLIENT_HTTP2", "on")
                # the ops port: /debug/state after the timed waves (each executor's client flow control, the
                # coordinator's GC passes); executors report their state every second
                import socket as _socket
                with _socket.socket() as _s:
                    _s.bind(("127.0.0.1", 0))
                    ops_port = _s.getsockname()[1]
                env.setdefault("NEXUS__HEALTH_BIND_ADDRESS", f"127.0.0.1:{ops_port}")
                env.setdefault("NCC_STATUS_S", "1")
                if args.stages:
                    env["NCC_TRACE_STAGES"] = os.path.join(work, "trace")
                    os.makedirs(env["NCC_TRACE_STAGES"], exist_ok=True)
                log = open(os.path.join(work, "controller.log"), "wb")
                t_boot = time.time_ns()
                controller = subprocess.Popen([sys.executable, "-m", "ncc"], env=env, stdout=log,
                                              stderr=subprocess.STDOUT, cwd=work)
                pin(controller, 0)  # before it starts its executors: they inherit the mask
                procs.append(controller)
            t_boot = d.broadcast(t_boot if d.rank == 0 else None)
            named = {"shard-apiserver": procs[0]}
            if d.rank == 0:
                named.update({"controller-apiserver": ctrl_proc, "coordinator": controller})

            total = args.warmup + args.steps
            if d.rank == 0:
                # every wave is sent and decoded by the controller apiserver before the clock starts; a
                # timed step commits a staged wave (the load generator's request is not the system under test)
                for v in range(1, total + 1):
                    await post(session, f"{ctrl_url}/_fake/stage", wave_body(T, v, args.payload, stage_id=v))
                    if total > 200 and v % 100 == 0:  # a long soak: a sign of life while it stages
                        print(f"# staged {v}/{total} waves", file=sys.stderr, flush=True)

            async def converge(version: int, times: bool, url=None):
                if url is None and S > 1:  # every shard this rank hosts; times keyed per shard
                    rs = await asyncio.gather(*(converge(version, times, u) for u in my_urls))
                    merged = {}
                    for j, r in enumerate(rs):
                        for marker, objs in (r.get("times") or {}).items():
                            merged.setdefault(marker, {}).update({f"{j}:{k}": t for k, t in objs.items()})
                    return {"ok": True, "times": merged}
                r = await post(session, f"{url or my_url}/_fake/markers/wait",
                               {"want": want(T, version), "timeout": args.timeout, "times": times, "keyed": True},
                               timeout=args.timeout + 30)
                if not r["ok"]:
                    tail = ""
                    if controller is not None:
                        with open(os.path.join(work, "controller.log"), "rb") as f:
                            tail = f.read()[-3000:].decode(errors="replace")
                    raise RuntimeError(f"rank {d.rank}: wave v{version} did not converge: {r['counts']}\n{tail}")
                return r

            # ---- cold start (warm-up 0): boot + full fan-out of pre-seeded objects
            r = await converge(0, True)
            d.barrier()
            cold_local = max(max(v.values()) for v in r["times"].values()) - t_boot
            cold = d.max(cold_local / 1e9)

            shard_times: list[dict] = []  # per timed wave: {"plural=value": {"ns/name": t_ns}}
            ctrl_times: list[dict] = []
            t_start = None
            t0s: dict = {}
            debug = bool(os.environ.get("NCC_BENCH_DEBUG"))
            for step in range(1, total + 1):
                if step == args.warmup + 1:
                    cg0 = cgroup_cpu()
                    cs0 = ctx_switches(named)
                    load0 = os.getloadavg()
                    hb0 = host_busy()
                    d.sync()
                    t_start = time.perf_counter()
                    sys0: dict = {}
                    cpu0 = cpu_seconds(named, sys_out=sys0)
                    kids0 = child_pids(controller) if controller is not None else set()
                    placement = Placement(named).start() if d.rank == 0 else None
                t0 = None
                if d.rank == 0:
                    a = await post(session, f"{ctrl_url}/_fake/apply", {"staged": step})
                    t0 = a["t0_ns"]
                    if debug:
                        print(f"# wave {step}: apply {(a['t1_ns'] - a['t0_ns']) / 1e6:.1f} ms", file=sys.stderr)
                t0 = t0s[step] = d.broadcast(t0)
                r = await converge(step, debug)
                if debug:
                    for plural, ts in r.get("times", {}).items():
                        ts = sorted(ts.values())
                        print(f"# wave {step} rank {d.rank} {plural}: first {(ts[0] - t0) / 1e6:.1f} "
                              f"p50 {(ts[len(ts) // 2] - t0) / 1e6:.1f} last {(ts[-1] - t0) / 1e6:.1f} ms",
                              file=sys.stderr)
                d.barrier()  # the wave is done only when every shard has converged
                if total > 200 and step % 100 == 0 and d.rank == 0:
                    print(f"# wave {step}/{total}", file=sys.stderr, flush=True)
            d.sync()
            elapsed = time.perf_counter() - t_start
            placed = placement.stop() if placement is not None else None
            rss: dict = {}
            sys1: dict = {}
            cpu1 = cpu_seconds(named, rss, sys1)
            cg1 = cgroup_cpu()
            cs1 = ctx_switches(named)
            load1 = os.getloadavg()
            hb1 = host_busy()
            ctrl_api = None
            ctrl_state = {}
            if d.rank == 0 and os.path.exists(os.path.join(work, "topology.json")):
                with open(os.path.join(work, "topology.json")) as f:
                    ctrl_state["sizing"] = json.load(f)
            ctl_debug = None
            if d.rank == 0:
                try:
                    await asyncio.sleep(1.2)  # one more status message from every executor, after the waves
                    async with session.get(f"http://{env['NEXUS__HEALTH_BIND_ADDRESS']}/debug/state",
                                           timeout=aiohttp.ClientTimeout(total=10)) as r:
                        st = await r.json()
                    flow = {}
                    for h in (st.get("executors") or {}).values():
                        flow.update((h.get("status") or {}).get("flow") or {})
                    ctl_debug = {"executor_flow": flow, "coordinator_gc": st.get("gc"),
                                 "controller_transport": st.get("controller_transport", "n/a")}
                except Exception as e:  # noqa: BLE001 — diagnostics only
                    ctl_debug = {"error": repr(e)[:200]}
            if d.rank == 0:  # LIST/WATCH load the controller put on its own cluster (watch relay: 1 each per kind)
                import aiohttp as _aiohttp
                async with session.get(f"{ctrl_url}/_fake/stats", timeout=_aiohttp.ClientTimeout(total=30)) as r:
                    st = await r.json()
                ctrl_api = {"lists": st["state"]["list"], "watches": st["state"]["watch"],
                            "requests": st["requests"]["total"]}
            kids1 = child_pids(controller) if controller is not None else set()
            util = {k: round((cpu1[k] - cpu0.get(k, 0.0)) / elapsed, 3) for k in cpu1}
            # Commit times stay on the servers (first time each object reached each version), so they are
            # fetched after the clock stops: shipping 3·T timestamps per wave is the load generator's work.
            for step in range(args.warmup + 1, total + 1):
                shard_times.append((await converge(step, True))["times"])
                if d.rank == 0:  # controller-side commit times of the same objects
                    ctrl_times.append((await converge(step, True, ctrl_url))["times"])
                    if debug:  # per kind: controller commits vs shard commits, ms after the wave's apply
                        for plural, ts in ctrl_times[-1].items():
                            c = sorted(ts.values())
                            sh = shard_times[-1].get(plural, {})
                            lt = sorted(t - ts[k.split(":", 1)[-1]] for k, t in sh.items())
                            print(f"# wave {step} {plural}: controller {(c[0] - t0s[step]) / 1e6:.1f}.."
                                  f"{(c[-1] - t0s[step]) / 1e6:.1f} ms, latency p50 {lt[len(lt) // 2] / 1e6:.1f} "
                                  f"max {lt[-1] / 1e6:.1f} ms", file=sys.stderr)
            utils = d.all_gather(util)
            # the shard apiserver's CPU per object it committed (the substrate's cost; every rank's shard
            # apiserver commits 3·T·steps objects per hosted shard)
            sub = (cpu1.get("shard-apiserver", 0.0) - cpu0.get("shard-apiserver", 0.0)) * 1e6 / (args.steps * 3 * T)
            subs = d.all_gather(sub)
            host = None
            if d.rank == 0:
                host = {"cpu_model": cpu_model(), "cpus": os.cpu_count(), "cgroup": cg1,
                        "throttled_usec": (cg1.get("throttled_usec", 0) - cg0.get("throttled_usec", 0))
                        if "throttled_usec" in cg1 else None,
                        "nr_throttled": (cg1.get("nr_throttled", 0) - cg0.get("nr_throttled", 0))
                        if "nr_throttled" in cg1 else None,
                        "loadavg": [round(x, 2) for x in load0] + [round(x, 2) for x in load1],
                        "ctx_switches": {k: [v[0] - cs0.get(k, [0, 0])[0], v[1] - cs0.get(k, [0, 0])[1]]
                                         for k, v in cs1.items()},
                        "placement": placed,
                        "pinned": {"controller": pin_sets[0], "apiservers": pin_sets[1] if args.pin == "l3" else None}
                        if pin_sets else None,
                        # CPUs the whole host kept busy over the timed waves (every tenant, this job included)
                        "host_busy_cpus": round((hb1[0] - hb0[0]) / elapsed, 1) if hb0 and hb1 else None,
                        "calibration": calibrate()}
            rsses = d.all_gather(rss)
            elapsed = d.max(elapsed)
            all_times = d.all_gather(shard_times)
            if d.rank != 0:
                return None
            lat = []  # per object and shard: shard commit − controller commit of the same version
            for per_rank in all_times:
                for wave, ctrl in zip(per_rank, ctrl_times):
                    for marker, objs in wave.items():
                        c = ctrl[marker]
                        lat.extend((t - c[k.split(":", 1)[-1]]) / 1e6 for k, t in objs.items())
            objs = args.steps * 3 * T * d.world * S
            value = objs / elapsed
            stages = None
            if args.stages:
                controller.terminate()  # the relay and the executors write their traces on shutdown
                try:
                    controller.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    pass
                stages = stage_breakdown(os.path.join(work, "trace"), ctrl_times, all_times[0])
            # controller CPU (coordinator + every executor, all on rank 0) per synced object over the timed
            # waves: the cost of the system under test, independent of how fast the fake apiservers are
            ctl_cpu = {k: cpu1.get(k, 0.0) - cpu0.get(k, 0.0) for k in ("coordinator", "executors")}
            us_per_obj = {k: round(v * 1e6 / objs, 1) for k, v in ctl_cpu.items()}
            # every hosted shard has its own apiserver process; `sub` is the first one's CPU per object it
            # committed, so the mean over ranks is already per object (no division by the shards per rank)
            substrate = sum(subs) / len(subs) if subs else None
            ctl_us = sum(ctl_cpu.values()) * 1e6 / objs
            from ncc.app import cpu_share
            sizing = ctrl_state.get("sizing") or {}
            ctrl_alive = controller.poll() is None
            return {
                "metric": METRIC,
                "value": round(value, 1),
                "unit": "objects/s",
                "n_gpus": d.world,
                "steps": args.steps,
                "warmup": args.warmup,
                "ms_per_step": round(elapsed * 1000 / args.steps, 2),
                "higher_is_better": True,
                "scaling": "weak",
                "vs_baseline": None,
                "dtype": "n/a",  # a control plane: no tensor arithmetic, so no numeric precision to report
                "data": "synthetic (fake kube-apiservers, random NexusAlgorithmTemplate/Secret/ConfigMap objects)",
                "config": {"model": "NexusAlgorithmTemplate fan-out (1 Secret + 1 ConfigMap each)",
                           "global_batch": T, "seq_len": 3, "parallelism": f"shards{d.world}",
                           "templates": T, "shards": d.world * S, "mode": args.mode, "payload_bytes": args.payload,
                           "shard_latency_ms": args.shard_latency_ms, "shard_jitter_ms": args.shard_jitter_ms,
                           "tls": bool(args.tls),
                           # what the C++ executors spoke to the shard apiservers and the coordinator to the
                           # controller apiserver (client-http2 on: HTTP/2 with prior knowledge to the shards; the
                           # controller cluster as client-go on cleartext, HTTP/1.1 — ncc/config.py controller_http2)
                           "shard_transport": _shard_transport(ctl_debug),
                           "controller_transport": (ctl_debug or {}).get("controller_transport", "n/a")},
                "p50_latency_ms": round(statistics.median(lat), 2) if lat else None,
                "p99_latency_ms": round(pct(lat, 99), 2) if lat else None,
                "controller_cpu_us_per_object": round(ctl_us, 1),
                "controller_cpu_us_per_object_split": us_per_obj,
                # the same for the fake shard apiserver (the substrate, mean over ranks), and the box-invariant
                # ratio: controller CPU per synced object over the substrate's CPU per committed object
                "substrate_us_per_object": round(substrate, 1) if substrate else None,
                "controller_to_substrate": round(ctl_us / substrate, 3) if substrate else None,
                "controller_to_substrate_split": {k: round(v / substrate, 3) for k, v in us_per_obj.items()}
                if substrate else None,
                "host": host,
                # per shard: the C++ executor's adaptive concurrency limit at the end, the most requests in flight,
                # 429s and overload signals seen (native/executor/http.hpp); the coordinator's GC passes
                "controller_state": ctl_debug,
                # kernel-mode share of that CPU (syscalls, the loopback TCP stack) per process
                "controller_cpu_sys_share": {k: round((sys1.get(k, 0.0) - sys0.get(k, 0.0)) / v, 3)
                                             for k, v in ctl_cpu.items() if v > 0},
                "cold_start_s": round(cold, 3),
                "cold_start_objects_per_s": round(3 * T * d.world * S / cold, 1) if cold > 0 else None,
                "controller_alive": ctrl_alive,
                # processes under the controller over the timed waves; a restarted child shows as replaced
                "controller_children": {"start": len(kids0), "end": len(kids1), "replaced": len(kids0 - kids1)},
                "controller_apiserver_load": ctrl_api,
                "controller_sizing": {"cpus": cpu_share(), **sizing,
                                      "overrides": [kv for kv in args.extra_env if kv.startswith(("NEXUS__", "NCC_"))]},
                # busy CPU cores per process over the timed steps (rank 0's, plus the busiest shard server)
                "cpu_cores_busy": dict(utils[0], **{"shard-apiserver-max": max(u.get("shard-apiserver", 0.0)
                                                                                 for u in utils)}),
                "rss_mib": dict(rsses[0], **{"shard-apiserver-max": max(r.get("shard-apiserver", 0.0)
                                                                       for r in rsses)}),
                **({"stages": stages} if stages is not None else {}),
            }
    finally:
        for p in reversed(procs):
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
        if not args.keep:
            shutil.rmtree(work, ignore_errors=True)


def main():
    args = parse_args()
    d = Dist()
    if d.world != args.gpus and d.world > 1:
        print(f"warning: --gpus {args.gpus} != WORLD_SIZE {d.world}; using WORLD_SIZE", file=sys.stderr)
    if d.world == 1 and args.gpus > 1:
        raise SystemExit("bench.py --gpus N>1 must be launched with torch.distributed.run --nproc-per-node N")
    # a SIGTERM (a `timeout` around the run) unwinds like an exception, so `run`'s cleanup stops the fake
    # apiservers and the controller instead of leaving the controller and its executors behind
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
    try:
        res = asyncio.run(run(args, d))
        if not (args.no_tls_run or args.tls or args.product_defaults or args.mode != "native"):
            # The production transport next to the headline (VERDICT r5 "next 7"): the same shape with
            # every apiserver on HTTPS (HTTP/2 negotiated by ALPN on every connection, the coordinator's included)
            # and the controller on the product's defaults — what a default Helm install runs.  The headline
            # itself keeps the bench's settings, named in `bench_settings`.
            import copy
            a2 = copy.copy(args)
            a2.tls, a2.product_defaults = True, True
            tls = asyncio.run(run(a2, d))
            if res is not None and tls is not None:
                res["tls_value"] = tls["value"]
                res["tls_p50_ms"] = tls["p50_latency_ms"]
                res["tls_p99_ms"] = tls["p99_latency_ms"]
                res["tls_controller_cpu_us_per_object"] = tls["controller_cpu_us_per_object"]
                res["tls_controller_cpu_us_per_object_split"] = tls["controller_cpu_us_per_object_split"]
                res["tls_controller_to_substrate"] = tls["controller_to_substrate"]
                res["tls_config"] = {"tls": True, "shard_transport": tls["config"]["shard_transport"],
                                     "controller_transport": tls["config"]["controller_transport"],
                                     "cpu_affinity": (tls.get("controller_sizing") or {}).get("cpu_affinity"),
                                     "settings": "product defaults (cpu-affinity none, client-http2 auto)",
                                     "ms_per_step": tls["ms_per_step"]}
    finally:
        d.close()
    if res is not None:
        if not args.product_defaults:
            res["bench_settings"] = {
                "NCC_CPU_AFFINITY": os.environ.get("NCC_CPU_AFFINITY", "l3"),
                "NEXUS__CLIENT_HTTP2": os.environ.get("NEXUS__CLIENT_HTTP2", "on"),
                "product_defaults": {"cpu_affinity": "none", "client_http2": "auto (HTTP/2 by ALPN on TLS; "
                                                                               "HTTP/1.1 on cleartext)"},
                "note": "the headline runs cleartext with the bench's settings; tls_* is a default install's "
                        "transport (see tls_config)"}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
