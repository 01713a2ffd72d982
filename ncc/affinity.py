"""Keep the coordinator and its shard executors on one L3 domain (an opt-in deployment knob).

The coordinator relays every watch line to its executors and folds every report they send back: the two
sides exchange cache lines all the time.  On a host whose CPUs span several L3 domains (an EPYC has one per
CCD), the kernel places them wherever it finds room, and moves them; the box measurements show two regimes for
the same tree and load — coordinator ≈ 9 and executors ≈ 11 µs per object when they share a domain, ≈ 12 and
≈ 14 when they do not — while pinning them to one domain held every run in the fast one (docs/BENCHMARKS_ARCHIVE.md,
`profiles/r4/r4v`, `r4w`, `r4z`, `r4ab`).

`NCC_CPU_AFFINITY` (Helm `controller.cpuAffinity`):

* `none` (the default): placement is left to the kernel.  A production controller syncs far below the rates
  where the regimes above differ, and a mask chosen on a shared host can later trap it next to a noisy tenant.
* `l3`: at start-up, in `App.build` — before the executors are spawned (they inherit the mask) and before the
  informers start, so it costs the propagation path nothing — the coordinator restricts every thread of its
  process to the least busy L3 domain among the CPUs it may run on, when that domain has room (four hardware
  threads per controller process).  Nothing changes when the allowed CPUs are already within one domain (a pod
  with a static CPU-manager cpuset, `bench.py --pin`), when no domain is big enough, or when the topology cannot
  be read.  The choice is not final: every `NCC_CPU_AFFINITY_RECHECK_S` seconds (default 30, 0: never) an idle
  controller re-samples the host, and when its domain is more than 80 % busy while another has clearly more idle
  capacity it moves itself and its children there (`Placement.recheck`).

`os.sched_setaffinity(pid, …)` on Linux sets one thread's mask, so every move here walks `/proc/<pid>/task`: the
threads a process already has (the event loop's executor pool, resolver threads) move with it.
"""
from __future__ import annotations

import asyncio
import logging
import os
import time

log = logging.getLogger("ncc.affinity")

SYS_CPU = "/sys/devices/system/cpu"
BUSY_MOVE = 0.8       # recheck: the current domain's busy share above which a move is considered ...
GAIN_MOVE = 1.25      # ... to a domain with at least this many times its idle capacity ...
GAIN_MIN_SHARE = 0.25  # ... and at least a quarter of a domain's CPUs more of it


def cpu_list(text: str) -> list[int]:
    """"0-3,8,10-11" -> [0, 1, 2, 3, 8, 10, 11]"""
    out: list[int] = []
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def l3_domains(allowed, sys_cpu: str = SYS_CPU) -> dict[int, list[int]] | None:
    """The allowed CPUs grouped by the L3 cache they share (keyed by the domain's lowest CPU)."""
    doms: dict[int, list[int]] = {}
    for c in sorted(allowed):
        try:
            with open(f"{sys_cpu}/cpu{c}/cache/index3/shared_cpu_list") as f:
                dom = min(cpu_list(f.read()))
        except (OSError, ValueError):
            return None
        doms.setdefault(dom, []).append(c)
    return doms


def stat_sample(stat: str = "/proc/stat") -> dict[int, tuple[int, int]]:
    """Per CPU: (busy jiffies, total jiffies) so far (host-wide: other tenants included)."""
    out = {}
    with open(stat) as f:
        for ln in f:
            if ln.startswith("cpu") and ln[3:4].isdigit():
                parts = ln.split()
                v = [int(x) for x in parts[1:]]
                out[int(parts[0][3:])] = (sum(v) - v[3] - (v[4] if len(v) > 4 else 0), sum(v))
    return out


def busy_between(a: dict, b: dict, cpus) -> dict[int, float]:
    busy = {}
    for c in cpus:
        if c in a and c in b and b[c][1] > a[c][1]:
            busy[c] = (b[c][0] - a[c][0]) / (b[c][1] - a[c][1])
    return busy


def cpu_busy(cpus, interval: float = 0.05, stat: str = "/proc/stat") -> dict[int, float]:
    """Busy share of each CPU over `interval` seconds (blocking: tools and tests; the app samples with
    `cpu_busy_async`)."""
    a = stat_sample(stat)
    time.sleep(interval)
    return busy_between(a, stat_sample(stat), cpus)


async def cpu_busy_async(cpus, interval: float = 0.05, stat: str = "/proc/stat") -> dict[int, float]:
    a = stat_sample(stat)
    await asyncio.sleep(interval)
    return busy_between(a, stat_sample(stat), cpus)


def choose(domains: dict[int, list[int]], busy: dict[int, float], min_cpus: int) -> list[int] | None:
    """The domain to run on: with at least `min_cpus` allowed CPUs, the most idle CPU capacity, then the least
    busy; None when the allowed CPUs are one domain already or none is big enough."""
    if len(domains) < 2:
        return None
    best, best_key = None, None
    for cpus in domains.values():
        if len(cpus) < min_cpus:
            continue
        load = sum(busy.get(c, 1.0) for c in cpus)
        key = (len(cpus) - load, -load)
        if best_key is None or key > best_key:
            best, best_key = cpus, key
    return best


def set_process_affinity(pid: int, cpus) -> int:
    """Restrict every thread of process `pid` (0: this one) to `cpus`; returns the threads moved.  Threads
    that exit meanwhile are skipped; the process's own call raises when even its main thread cannot move."""
    proc = "self" if pid == 0 else str(pid)
    try:
        tids = [int(t) for t in os.listdir(f"/proc/{proc}/task")]
    except (OSError, ValueError):
        tids = []
    main = os.getpid() if pid == 0 else pid
    if main not in tids:
        tids.append(main)
    moved = 0
    for tid in tids:
        try:
            os.sched_setaffinity(tid, cpus)
            moved += 1
        except OSError:
            if tid == main:
                raise
    return moved


def policy_from_env(policy: str | None = None) -> str:
    return (policy if policy is not None else os.environ.get("NCC_CPU_AFFINITY", "none")).strip().lower()


class Placement:
    """The L3 domain this coordinator chose, and the processes on it.  `recheck` moves them all to another
    domain when the chosen one has filled up with other tenants' work."""

    def __init__(self, domains: dict[int, list[int]], cpus: list[int], processes: int):
        self.domains, self.cpus, self.processes = domains, list(cpus), processes
        self.moves = 0
        self.checks = 0

    def target(self, busy: dict[int, float]) -> list[int] | None:
        """Where to go now, or None to stay: the current domain more than BUSY_MOVE busy (over its CPUs) and
        the best domain with GAIN_MOVE times its idle capacity and GAIN_MIN_SHARE of a domain more."""
        cur = self.cpus
        cur_busy = sum(busy.get(c, 1.0) for c in cur) / max(1, len(cur))
        if cur_busy <= BUSY_MOVE:
            return None
        best = choose(self.domains, busy, min_cpus=max(8, 4 * self.processes))
        if best is None or best == cur:
            return None
        idle_cur = len(cur) - cur_busy * len(cur)
        idle_best = len(best) - sum(busy.get(c, 1.0) for c in best)
        if idle_best < GAIN_MOVE * max(idle_cur, 0.5) or idle_best - idle_cur < GAIN_MIN_SHARE * len(best):
            return None
        return best

    def move(self, cpus: list[int], pids) -> None:
        set_process_affinity(0, cpus)
        for pid in pids:
            try:
                set_process_affinity(pid, cpus)
            except OSError:  # a child that exited meanwhile (the pool respawns it from our new mask)
                pass
        log.warning("controller processes moved to another L3 domain: CPUs %s (the previous one was busy)", cpus)
        self.cpus = list(cpus)
        self.moves += 1

    async def recheck(self, pids, interval: float = 0.5) -> bool:
        self.checks += 1
        busy = await cpu_busy_async([c for cs in self.domains.values() for c in cs], interval)
        to = self.target(busy)
        if to is None:
            return False
        self.move(to, pids())
        return True

    async def loop(self, period: float, pids, idle) -> None:
        """Every `period` seconds, when `idle()` (the controller's queue is drained: its own load does not
        count against its domain), `recheck`."""
        while True:
            await asyncio.sleep(period)
            if idle is None or idle():
                try:
                    await self.recheck(pids)
                except (OSError, ValueError) as e:
                    log.debug("placement recheck failed: %s", e)


async def apply_async(processes: int, policy: str | None = None, interval: float = 0.05) -> Placement | None:
    """Restrict this process (every thread of it, and the children it starts afterwards) to one L3 domain with
    room for `processes` busy processes — four hardware threads each, so the shard apiservers and other tenants
    the kernel also puts there leave them a core: with 4 shards' executors squeezed into one 16-thread domain the
    box ran 12 % slower than unplaced (`profiles/r4/r4ag`), so larger groups are left to the kernel; returns
    the placement, or None when nothing changed."""
    policy = policy_from_env(policy)
    if policy in ("", "none", "0", "off"):
        return None
    if policy != "l3":
        log.warning("NCC_CPU_AFFINITY=%r: not one of l3, none; leaving the CPU mask alone", policy)
        return None
    try:
        allowed = os.sched_getaffinity(0)
    except (AttributeError, OSError):
        return None
    doms = l3_domains(allowed)
    if not doms or len(doms) < 2:
        return None
    try:
        busy = await cpu_busy_async(allowed, interval)
    except (OSError, ValueError):
        busy = {}
    cpus = choose(doms, busy, min_cpus=max(8, 4 * processes))
    if cpus is None:
        return None
    try:
        set_process_affinity(0, cpus)
    except OSError as e:
        log.warning("could not restrict the controller to one L3 domain: %s", e)
        return None
    log.info("controller processes on one L3 domain: CPUs %s (%d processes)", cpus, processes)
    return Placement(doms, cpus, processes)


def apply(processes: int, policy: str | None = None) -> list[int] | None:
    """Blocking `apply_async` (no running event loop): the CPUs chosen, or None."""
    p = asyncio.run(apply_async(processes, policy))
    return p.cpus if p is not None else None
