#!/usr/bin/env python
"""CPU cost of the executor's reconcile logic alone: `sync_template` in executor role against shard clients
that answer writes instantly (no network, no apiserver), with slim shard caches and the write-through
overlay, exactly as configured in native mode.  Reports µs per template pass (3 objects written).

    python scripts/micro_reconcile.py [--templates 2000] [--repeats 5]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ncc.api import resources as R  # noqa: E402
from ncc.cache.informer import Informer  # noqa: E402
from ncc.controller.controller import Controller  # noqa: E402
from ncc.controller.events import FakeRecorder  # noqa: E402
from ncc.controller.options import ControllerOptions  # noqa: E402
from ncc.controller.reconcile import slim_data, slim_spec  # noqa: E402
from ncc.shards.shard import Shard  # noqa: E402
from ncc.testing.workload import (configmap_name, make_configmap, make_secret, make_template,  # noqa: E402
                                  secret_name)

NS = "nexus"


class InstantClient:
    """Answers write_meta at once with a fresh resourceVersion; lists are empty."""
    cluster_name = "shard"

    def __init__(self):
        self.rv = 1000
        self.writes = 0

    async def list(self, rt, ns, **kw):
        return {"items": [], "metadata": {"resourceVersion": "1"}}

    async def write_meta(self, verb, rt, namespace, body, *, name=None, field_manager=None, patch_type=None,
                         force=None):
        self.rv += 1
        self.writes += 1
        m = body.get("metadata") or {}
        return namespace, name or m.get("name", ""), str(self.rv), m.get("uid") or f"uid-{self.rv}"

    async def close(self):
        pass


def build(n: int):
    opts = ControllerOptions.native(native_queue=True, role="executor")
    cclient = InstantClient()
    infs = {rt: Informer(cclient, rt, NS) for rt in (R.TEMPLATES, R.WORKGROUPS, R.SECRETS, R.CONFIGMAPS)}
    slim = {R.TEMPLATES: slim_spec, R.WORKGROUPS: slim_spec, R.SECRETS: slim_data, R.CONFIGMAPS: slim_data}
    sclient = InstantClient()
    shard = Shard("ctl", "shard-0", sclient, NS, assume_writes=True, sync_binary_data=True, transforms=slim)
    ctl = Controller(alias="ctl", namespace=NS, client=cclient, shards=[shard],
                     template_informer=infs[R.TEMPLATES], workgroup_informer=infs[R.WORKGROUPS],
                     secret_informer=infs[R.SECRETS], configmap_informer=infs[R.CONFIGMAPS], options=opts,
                     recorder=FakeRecorder(keep=False), shard_names=["shard-0"])
    ctl.reporter = lambda msg: None
    rv = 1
    for i in range(n):
        for obj, inf in ((make_secret(secret_name(i), NS), infs[R.SECRETS]),
                         (make_configmap(configmap_name(i), NS), infs[R.CONFIGMAPS]),
                         (make_template(i, NS, secrets=[secret_name(i)], configmaps=[configmap_name(i)]),
                          infs[R.TEMPLATES])):
            rv += 1
            obj["metadata"].update(resourceVersion=str(rv), uid=f"c-{rv}")
            inf.store.upsert(obj)
    for inf in list(infs.values()) + shard.factory.informers():
        inf._synced.set()
    return ctl, sclient


def bump(ctl, n: int, version: int):
    """A new version of every controller object (what a bench wave delivers)."""
    for i in range(n):
        for inf, name in ((ctl.secret_informer, secret_name(i)), (ctl.configmap_informer, configmap_name(i))):
            o = dict(inf.store.get(NS, name))
            o["data"] = {"version": str(version)}
            inf.store.upsert(o)
        t = ctl.template_informer.store.get(NS, f"algo-{i:05d}")
        t = dict(t, spec=dict(t["spec"], container=dict(t["spec"]["container"], versionTag=f"v{version}")))
        ctl.template_informer.store.upsert(t)


async def run(n: int, repeats: int) -> dict:
    ctl, sclient = build(n)
    for i in range(n):  # cold pass: creates everything
        await ctl.sync_template(NS, f"algo-{i:05d}")
    best = None
    for v in range(repeats):
        bump(ctl, n, v + 2)
        w0 = sclient.writes
        t0 = time.process_time()
        for i in range(n):
            await ctl.sync_template(NS, f"algo-{i:05d}")
        dt = time.process_time() - t0
        assert sclient.writes - w0 == 3 * n, (sclient.writes - w0, 3 * n)
        best = dt if best is None else min(best, dt)
    # a no-op pass: nothing changed
    t0 = time.process_time()
    for i in range(n):
        await ctl.sync_template(NS, f"algo-{i:05d}")
    noop = time.process_time() - t0
    return {"us_per_template_pass": round(best / n * 1e6, 2), "us_per_object": round(best / n / 3 * 1e6, 2),
            "us_per_noop_pass": round(noop / n * 1e6, 2)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--templates", type=int, default=2000)
    ap.add_argument("--repeats", type=int, default=5)
    a = ap.parse_args(argv)
    print(json.dumps(asyncio.run(run(a.templates, a.repeats))))
    return 0


if __name__ == "__main__":
    sys.exit(main())
