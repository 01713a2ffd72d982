"""Keep the coordinator and its shard executors on one L3 domain.

The coordinator relays every watch line to its executors and folds every report they send back: the two
sides exchange cache lines all the time.  On a host whose CPUs span several L3 domains (an EPYC has one per
CCD), the kernel places them wherever it finds room, and moves them; the box measurements show two regimes for
the same tree and load — coordinator ≈ 9 and executors ≈ 11 µs per object when they share a domain, ≈ 12 and
≈ 14 when they do not — while pinning them to one domain held every run in the fast one (BENCHMARKS.md
"Round 4", `profiles/r4/r4v`, `r4w`, `r4z`, `r4ab`).

At start-up, before the executors are spawned (they inherit the mask), the coordinator restricts itself to the
least busy L3 domain among the CPUs it may run on, when that domain has room for it
(`NCC_CPU_AFFINITY`: `l3`, the default, or `none`).  Nothing changes when the allowed CPUs are already within
one domain (a static CPU-manager pod, `bench.py --pin`), when no domain has at least `min_cpus` of them, or
when the topology cannot be read.
"""
from __future__ import annotations

import logging
import os
import time

log = logging.getLogger("ncc.affinity")

SYS_CPU = "/sys/devices/system/cpu"


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


def cpu_busy(cpus, interval: float = 0.05, stat: str = "/proc/stat") -> dict[int, float]:
    """Busy share of each CPU over `interval` seconds (host-wide /proc/stat: other tenants included)."""
    def sample():
        out = {}
        with open(stat) as f:
            for ln in f:
                if ln.startswith("cpu") and ln[3:4].isdigit():
                    parts = ln.split()
                    v = [int(x) for x in parts[1:]]
                    out[int(parts[0][3:])] = (sum(v) - v[3] - (v[4] if len(v) > 4 else 0), sum(v))
        return out
    a = sample()
    time.sleep(interval)
    b = sample()
    busy = {}
    for c in cpus:
        if c in a and c in b and b[c][1] > a[c][1]:
            busy[c] = (b[c][0] - a[c][0]) / (b[c][1] - a[c][1])
    return busy


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


def apply(processes: int, policy: str | None = None) -> list[int] | None:
    """Restrict this process (and the children it starts afterwards) to one L3 domain with room for
    `processes` busy processes — four hardware threads each, so the shard apiservers and other tenants the
    kernel also puts there leave them a core: with 4 shards' executors squeezed into one 16-thread domain the
    box ran 12 % slower than unplaced (`profiles/r4/r4ag`), so larger groups are left to the kernel; returns
    the CPUs chosen, or None when nothing changed."""
    policy = (policy if policy is not None else os.environ.get("NCC_CPU_AFFINITY", "l3")).strip().lower()
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
        busy = cpu_busy(allowed)
    except (OSError, ValueError):
        busy = {}
    cpus = choose(doms, busy, min_cpus=max(8, 4 * processes))
    if cpus is None:
        return None
    try:
        os.sched_setaffinity(0, cpus)
    except OSError as e:
        log.warning("could not restrict the controller to one L3 domain: %s", e)
        return None
    log.info("controller processes on one L3 domain: CPUs %s (%d processes)", cpus, processes)
    return cpus
