"""Per-component resource accounting of a running controller, for benchmarks at scale.

`ProcTree` samples the controller's process tree — the coordinator (`python -m ncc`), its C++ shard executors
(`ncc/bin/ncc-executor`) and any coordinator partitions (`python -m ncc --control-fd`) — and keeps, per
component, the current and peak resident set and the CPU seconds spent.  `Cgroup` runs the controller under a
CPU quota and a memory limit (cgroup v1 `cpu` + `memory` controllers, or v2 `cpu.max` + `memory.max`) and
reads back what the kernel saw: peak usage, limit hits, OOM kills, throttling.  Both answer VERDICT r5
"next 1": does the controller fit the reference chart's suggested 1 CPU / 1 GiB
(/root/reference/.helm/values.yaml:113-122) at BASELINE config 4's 8 shards × 10 000 templates?
"""
from __future__ import annotations

import asyncio
import os
import time

ROLES = ("coordinator", "executors", "partitions", "other")


def classify(proc, root_pid: int) -> str:
    if proc.pid == root_pid:
        return "coordinator"
    try:
        name = proc.name()
        cmd = proc.cmdline()
    except Exception:  # noqa: BLE001 — gone between listing and reading
        return "other"
    if name.startswith("ncc-executor") or any(c.endswith("ncc-executor") for c in cmd[:1]):
        return "executors"
    if "--control-fd" in cmd:
        return "partitions"
    return "other"


class ProcTree:
    """Samples a process and its descendants every `period` seconds (`start()`/`stop()`), or on demand."""

    def __init__(self, pid: int, period: float = 0.2):
        import psutil
        self._psutil = psutil
        self.root_pid = pid
        self.period = period
        self.procs: dict[int, tuple] = {}  # pid -> (psutil.Process, role)
        self.peak = {r: 0 for r in ROLES}
        self.peak["total"] = 0
        self.cpu_last: dict[int, float] = {}  # pid -> last cpu seconds seen (children that exited keep theirs)
        self.cpu_role = {r: 0.0 for r in ROLES}
        self.counts = {r: 0 for r in ROLES}
        self.samples = 0
        self._task = None
        self._marks: dict[str, dict] = {}

    def _refresh(self) -> None:
        psutil = self._psutil
        try:
            root = psutil.Process(self.root_pid)
            tree = [root] + root.children(recursive=True)
        except psutil.Error:
            return
        seen = set()
        for p in tree:
            seen.add(p.pid)
            if p.pid not in self.procs:
                self.procs[p.pid] = (p, classify(p, self.root_pid))
        for pid in list(self.procs):
            if pid not in seen:
                self.procs.pop(pid)

    def sample(self) -> dict:
        """{role: current RSS bytes}, updating peaks and CPU seconds."""
        self._refresh()
        cur = {r: 0 for r in ROLES}
        counts = {r: 0 for r in ROLES}
        for pid, (p, role) in list(self.procs.items()):
            try:
                with p.oneshot():
                    rss = p.memory_info().rss
                    t = p.cpu_times()
                cpu = t.user + t.system
            except self._psutil.Error:
                continue
            cur[role] += rss
            counts[role] += 1
            prev = self.cpu_last.get(pid, 0.0)
            if cpu > prev:
                self.cpu_role[role] += cpu - prev
                self.cpu_last[pid] = cpu
        total = sum(cur.values())
        for r in ROLES:
            self.peak[r] = max(self.peak[r], cur[r])
        self.peak["total"] = max(self.peak["total"], total)
        self.counts = {r: max(self.counts[r], counts[r]) for r in ROLES}
        self.samples += 1
        cur["total"] = total
        return cur

    async def _loop(self) -> None:
        while True:
            self.sample()
            await asyncio.sleep(self.period)

    def start(self) -> "ProcTree":
        self._task = asyncio.ensure_future(self._loop())
        return self

    async def stop(self) -> None:
        if self._task is not None:
            self._task.cancel()
            await asyncio.gather(self._task, return_exceptions=True)
            self._task = None
        self.sample()

    def reset_peaks(self) -> None:
        """Peaks from now on (a phase's own peak)."""
        cur = self.sample()
        for r in ROLES + ("total",):
            self.peak[r] = cur[r]

    def mark(self, name: str) -> None:
        """Remember CPU seconds and wall time now; `since(name)` reports what was spent after it."""
        self.sample()
        self._marks[name] = {"t": time.perf_counter(), "cpu": dict(self.cpu_role)}

    def since(self, name: str) -> dict:
        self.sample()
        m = self._marks[name]
        wall = time.perf_counter() - m["t"]
        cpu = {r: round(self.cpu_role[r] - m["cpu"][r], 3) for r in ROLES if self.counts[r]}
        return {"wall_s": round(wall, 3), "cpu_s": cpu, "cpu_s_total": round(sum(cpu.values()), 3),
                "cores_busy": round(sum(cpu.values()) / wall, 3) if wall > 0 else None}

    def report(self) -> dict:
        mib = 1 << 20
        return {"processes": {r: n for r, n in self.counts.items() if n},
                "peak_rss_mib": {r: round(v / mib, 1) for r, v in self.peak.items() if v},
                "cpu_s": {r: round(v, 3) for r, v in self.cpu_role.items() if self.counts[r]},
                "samples": self.samples}


class Cgroup:
    """A throwaway cgroup with a CPU quota and a memory limit (needs write access to the cgroup mounts:
    root in a container, or a delegated v2 subtree).  `available()` says whether one can be made here."""

    V1 = "/sys/fs/cgroup"

    def __init__(self, name: str, cpus: float, memory_bytes: int):
        self.name = name
        self.cpus = cpus
        self.memory_bytes = memory_bytes
        self.dirs: dict[str, str] = {}
        self.version = 0

    @staticmethod
    def available() -> bool:
        v1 = all(os.access(os.path.join(Cgroup.V1, c), os.W_OK) for c in ("cpu", "memory"))
        v2 = os.path.exists(os.path.join(Cgroup.V1, "cgroup.controllers")) and os.access(Cgroup.V1, os.W_OK)
        return v1 or v2

    def create(self) -> "Cgroup":
        period = 100000
        quota = int(self.cpus * period)
        if os.path.isdir(os.path.join(self.V1, "cpu")) and os.path.isdir(os.path.join(self.V1, "memory")):
            self.version = 1
            for c in ("cpu", "memory"):
                d = os.path.join(self.V1, c, self.name)
                os.makedirs(d, exist_ok=True)
                self.dirs[c] = d
            self._write("cpu", "cpu.cfs_period_us", period)
            self._write("cpu", "cpu.cfs_quota_us", quota)
            self._write("memory", "memory.limit_in_bytes", self.memory_bytes)
            try:  # no swap to spill into: the limit is the limit
                self._write("memory", "memory.memsw.limit_in_bytes", self.memory_bytes)
            except OSError:
                pass
        else:
            self.version = 2
            d = os.path.join(self.V1, self.name)
            os.makedirs(d, exist_ok=True)
            self.dirs = {"cpu": d, "memory": d}
            self._write("cpu", "cpu.max", f"{quota} {period}")
            self._write("memory", "memory.max", self.memory_bytes)
            try:
                self._write("memory", "memory.swap.max", 0)
            except OSError:
                pass
        return self

    def _write(self, c: str, f: str, v) -> None:
        with open(os.path.join(self.dirs[c], f), "w") as fh:
            fh.write(str(v))

    def _read(self, c: str, f: str) -> str:
        try:
            with open(os.path.join(self.dirs[c], f)) as fh:
                return fh.read()
        except OSError:
            return ""

    def enter(self) -> None:
        """Move the calling process into the cgroup (a `preexec_fn`: the child and everything it spawns)."""
        pid = str(os.getpid())
        for d in dict.fromkeys(self.dirs.values()):
            with open(os.path.join(d, "cgroup.procs"), "w") as fh:
                fh.write(pid)

    def stats(self) -> dict:
        def kv(text):
            out = {}
            for line in text.splitlines():
                k, _, v = line.partition(" ")
                try:
                    out[k] = int(v)
                except ValueError:
                    pass
            return out
        mib = 1 << 20
        out = {"cgroup_version": self.version, "cpus": self.cpus, "memory_limit_mib": round(self.memory_bytes / mib)}
        cpu = kv(self._read("cpu", "cpu.stat"))
        if self.version == 1:
            peak = self._read("memory", "memory.max_usage_in_bytes").strip()
            usage = self._read("memory", "memory.usage_in_bytes").strip()
            oom = kv(self._read("memory", "memory.oom_control"))
            mstat = kv(self._read("memory", "memory.stat"))
            out.update(peak_mib=round(int(peak or 0) / mib, 1), usage_mib=round(int(usage or 0) / mib, 1),
                       limit_hits=int(self._read("memory", "memory.failcnt").strip() or 0),
                       oom_kills=oom.get("oom_kill", 0),
                       rss_mib=round(mstat.get("total_rss", mstat.get("rss", 0)) / mib, 1),
                       cache_mib=round(mstat.get("total_cache", mstat.get("cache", 0)) / mib, 1),
                       nr_periods=cpu.get("nr_periods", 0), nr_throttled=cpu.get("nr_throttled", 0),
                       throttled_s=round(cpu.get("throttled_time", 0) / 1e9, 3))
        else:
            ev = kv(self._read("memory", "memory.events"))
            peak = self._read("memory", "memory.peak").strip()
            usage = self._read("memory", "memory.current").strip()
            out.update(peak_mib=round(int(peak or 0) / mib, 1) if peak else None,
                       usage_mib=round(int(usage or 0) / mib, 1), limit_hits=ev.get("max", 0),
                       oom_kills=ev.get("oom_kill", 0), nr_periods=cpu.get("nr_periods", 0),
                       nr_throttled=cpu.get("nr_throttled", 0), throttled_s=round(cpu.get("throttled_usec", 0) / 1e6, 3))
        return out

    def remove(self) -> None:
        for d in dict.fromkeys(self.dirs.values()):
            for _ in range(50):
                try:
                    os.rmdir(d)
                    break
                except OSError:
                    time.sleep(0.1)
