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
def test_apply_restricts_to_the_chosen_domain(monkeypatch, tmp_path):
    doms = {0: list(range(12)), 12: list(range(12, 24))}
    monkeypatch.setattr(affinity, "l3_domains", lambda allowed: doms)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(24)))
    monkeypatch.setattr(affinity, "cpu_busy", lambda cpus: {c: (0.8 if c < 12 else 0.0) for c in cpus})
    got = []
    monkeypatch.setattr(os, "sched_setaffinity", lambda pid, cpus: got.append(list(cpus)))
    assert affinity.apply(3, "l3") == list(range(12, 24))  # 3 processes: 12 threads
    assert got == [list(range(12, 24))]
    assert affinity.apply(4, "l3") is None  # 4 processes need 16 threads: no domain has room
