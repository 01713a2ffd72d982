"""BASELINE config 4 at reduced scale (VERDICT r5 "next 1"): 2 000 templates × 4 shards, cold-start adoption of
pre-existing shard objects, two steady-state waves, then a relist storm on all five apiservers at once
(`/_fake/faults {"relist": true}`: the watch history compacted past every client's revision and every watch
dropped — each informer of the controller, coordinator and C++ executors alike, must relist).

Asserted:
* the storm issues no write at all — not on the shards, not on the controller cluster (no status, adoption or
  Event write) — and the coordinator runs no template pass: every object is already in sync, so a relist must
  be read-only.  The reference gets the same relist
  from client-go's reflector (/root/reference/main.go:70-71, controller.go:862-871), and re-reconciles every
  template after it (its handlers enqueue every update);
* every watch is back (and relisted) within the timeout, and an update wave after the storm still converges;
* a resident-set bound per cached object: the controller's processes (coordinator + executors) settle below
  16 KiB per object they cache — 3 objects per template on the controller cluster and on each shard.

The full-scale run (10 000 × 8, and under a 1 CPU / 1 GiB cgroup) is `bench/suite.py --configs 4`
(BENCHMARKS.md "Config 4 at scale").
"""
import asyncio
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.slow
def test_relist_storm_is_read_only_and_memory_is_bounded():
    from ncc.controller.native_executor import binary_path
    if binary_path() is None:
        pytest.skip("the C++ executor is not built")
    sys.path.insert(0, os.path.join(ROOT, "bench"))
    import suite
    T, shards = 2000, 4
    r = asyncio.run(suite.config4_adoption("native", T, timeout=240, n_shards=shards, waves=2, storm=True))
    assert r["ok"] and r.get("all_ready"), r.get("log_tail") or r.get("counts")
    assert r["objects_written"] > 0  # the cold start did adopt and fix the pre-existing shard objects
    assert r["waves"]["ok"]
    st = r["relist_storm"]
    assert st["ok"], st
    assert st["relists"] >= st["watches_dropped"] > 0
    assert st["shard_writes"] == 0 and st["controller_writes"] == 0, st["writes_by_request"]
    # and reconciles nothing: a relisted object at the version already cached is no event (round 6 fix: an
    # adoption's echo skipped as "owners unchanged" left the pre-adoption version in the metadata-only store, so
    # every relist re-enqueued every template)
    assert st["coordinator_passes"] == {"reconciles": 0, "inline_finishes": 0}, st["coordinator_passes"]
    assert st["wave_after"]["ok"], st
    assert r["controller_alive"]
    settled = r["resources"]["phases"]["settled"]["rss_mib"]["total"]
    cached = 3 * T * (1 + shards)
    assert settled * 2**20 / cached < 16 * 1024, (settled, r["resources"])
