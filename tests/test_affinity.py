"""ncc/affinity.py: the coordinator's choice of one L3 domain for itself and its executors."""
import os

import pytest

from ncc import affinity


def _fake_sys(tmp_path, doms):
    """A /sys/devices/system/cpu tree whose L3 domains are `doms` (lists of CPUs)."""
    for cpus in doms:
        text = ",".join(str(c) for c in cpus)
        for c in cpus:
            d = tmp_path / f"cpu{c}" / "cache" / "index3"
            d.mkdir(parents=True)
            (d / "shared_cpu_list").write_text(text + "\n")
    return str(tmp_path)


def test_cpu_list():
    assert affinity.cpu_list("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert affinity.cpu_list("") == []


def test_domains_group_allowed_cpus(tmp_path):
    sys_cpu = _fake_sys(tmp_path, [[0, 1, 2, 3], [4, 5, 6, 7]])
    assert affinity.l3_domains({1, 2, 5}, sys_cpu) == {0: [1, 2], 4: [5]}
    assert affinity.l3_domains({9}, sys_cpu) is None  # unreadable topology: leave the mask alone


def test_choose_prefers_idle_capacity_and_skips_small_domains():
    doms = {0: [0, 1, 2, 3], 4: [4, 5, 6, 7], 8: [8, 9]}
    busy = {c: 0.9 for c in range(4)} | {c: 0.1 for c in range(4, 10)}
    assert affinity.choose(doms, busy, min_cpus=4) == [4, 5, 6, 7]
    assert affinity.choose(doms, busy, min_cpus=5) is None     # no domain has room
    assert affinity.choose({0: [0, 1, 2, 3]}, busy, 2) is None  # already one domain


def test_policy_none_and_unknown_leave_the_mask(monkeypatch):
    calls = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda *a: calls.append(a), raising=False)
    assert affinity.apply(3, "none") is None
    assert affinity.apply(3, "numa") is None
    assert calls == []


@pytest.mark.skipif(not hasattr(os, "sched_getaffinity"), reason="Linux only")
def test_apply_restricts_every_thread_to_the_chosen_domain(monkeypatch, tmp_path):
    """A pod whose cpuset spans several domains is pinned to one — every thread of the process."""
    doms = {0: list(range(12)), 12: list(range(12, 24))}
    monkeypatch.setattr(affinity, "l3_domains", lambda allowed: doms)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(24)))
    monkeypatch.setattr(affinity, "stat_sample", lambda stat="/proc/stat": {})
    monkeypatch.setattr(affinity, "busy_between", lambda a, b, cpus: {c: (0.8 if c < 12 else 0.0) for c in cpus})
    got = {}
    monkeypatch.setattr(os, "sched_setaffinity", lambda tid, cpus: got.__setitem__(tid, list(cpus)))
    assert affinity.apply(3, "l3") == list(range(12, 24))  # 3 processes: 12 threads
    tids = {int(t) for t in os.listdir("/proc/self/task")}
    assert os.getpid() in got and set(got) <= tids | {os.getpid()}
    assert all(v == list(range(12, 24)) for v in got.values())
    got.clear()
    assert affinity.apply(4, "l3") is None  # 4 processes need 16 threads: no domain has room
    assert got == {}


@pytest.mark.skipif(not hasattr(os, "sched_getaffinity"), reason="Linux only")
def test_pod_within_one_domain_is_left_alone(monkeypatch, tmp_path):
    """A pod whose cpuset is one L3 domain (a static CPU-manager allocation) keeps its mask."""
    sys_cpu = _fake_sys(tmp_path, [[0, 1, 2, 3, 4, 5, 6, 7], [8, 9, 10, 11, 12, 13, 14, 15]])
    real = affinity.l3_domains
    monkeypatch.setattr(affinity, "l3_domains", lambda allowed: real(allowed, sys_cpu))
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(8, 16)))
    calls = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda *a: calls.append(a))
    assert affinity.apply(1, "l3") is None and calls == []
    # ... while one spanning both domains is pinned to the idler one
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(16)))
    monkeypatch.setattr(affinity, "busy_between", lambda a, b, cpus: {c: (0.9 if c < 8 else 0.1) for c in cpus})
    assert affinity.apply(1, "l3") == list(range(8, 16)) and calls


def test_default_policy_is_none(monkeypatch):
    monkeypatch.delenv("NCC_CPU_AFFINITY", raising=False)
    assert affinity.policy_from_env() == "none"
    monkeypatch.setenv("NCC_CPU_AFFINITY", " L3 ")
    assert affinity.policy_from_env() == "l3"


def test_recheck_moves_off_a_busy_domain_only_with_a_clear_gain(monkeypatch):
    doms = {0: list(range(8)), 8: list(range(8, 16)), 16: list(range(16, 24))}
    p = affinity.Placement(doms, list(range(8)), processes=2)
    calm = {c: 0.5 for c in range(24)}
    assert p.target(calm) is None                                   # our domain is not full
    busy = {c: (0.95 if c < 8 else 0.9) for c in range(24)}
    assert p.target(busy) is None                                   # everyone is busy: no gain in moving
    busy.update({c: 0.1 for c in range(16, 24)})
    assert p.target(busy) == list(range(16, 24))
    moved = []
    monkeypatch.setattr(affinity, "set_process_affinity", lambda pid, cpus: moved.append((pid, list(cpus))))
    p.move(list(range(16, 24)), [111, 222])
    assert [m[0] for m in moved] == [0, 111, 222] and p.cpus == list(range(16, 24)) and p.moves == 1


async def test_recheck_loop_waits_for_idle(monkeypatch):
    import asyncio
    doms = {0: list(range(8)), 8: list(range(8, 16))}
    p = affinity.Placement(doms, list(range(8)), processes=1)
    checks = []

    async def recheck(pids, interval=0.5):
        checks.append(pids())
        return False
    monkeypatch.setattr(p, "recheck", recheck)
    idle = [False]
    t = asyncio.ensure_future(p.loop(0.01, lambda: [1], lambda: idle[0]))
    await asyncio.sleep(0.05)
    assert checks == []
    idle[0] = True
    await asyncio.sleep(0.05)
    t.cancel()
    assert checks and checks[0] == [1]
