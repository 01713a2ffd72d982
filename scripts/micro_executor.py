#!/usr/bin/env python
"""Per-operation CPU costs of the executor's hot paths, in one process, for directing optimisation work.

Measures client-side CPU (time.process_time) per unit of work, min over repeats:
  * informer watch lines: dropped by the partition filter / echo of our own write / decoded + dispatched
  * one shard write (PUT via write_meta, slim publish) against a fake apiserver in a child process, and
    that apiserver's own CPU per write

    python scripts/micro_executor.py [--lines 30000] [--writes 20000] [--repeats 5]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ncc.api import resources as R  # noqa: E402
from ncc.cache.informer import Informer  # noqa: E402
from ncc.controller.executor import key_part, partition_owner_filter  # noqa: E402
from ncc.testing.workload import make_secret  # noqa: E402

NS = "nexus"


def secret_lines(n: int, rv0: int = 1000) -> list[bytes]:
    out = []
    for i in range(n):
        s = make_secret(f"sec-{i:05d}", NS, payload=512, version=3)
        s["metadata"].update(resourceVersion=str(rv0 + i), uid=f"u{i}", ownerReferences=[
            {"apiVersion": "science.sneaksanddata.com/v1", "kind": "NexusAlgorithmTemplate",
             "name": f"algo-{i:05d}", "uid": f"t{i}"}])
        out.append(json.dumps({"type": "MODIFIED", "object": s}, separators=(",", ":")).encode())
    return out


class _LinesClient:
    cluster_name = "micro"

    def __init__(self, lines):
        self.lines = lines

    async def list(self, rt, ns, **kw):
        return {"items": [], "metadata": {"resourceVersion": "1"}}

    async def watch_raw(self, rt, ns, **kw):  # pragma: no cover - batches are used
        for ln in self.lines:
            yield ln

    async def watch_raw_batches(self, rt, ns, **kw):
        for j in range(0, len(self.lines), 100):
            yield self.lines[j:j + 100]
            await asyncio.sleep(0)


async def informer_case(lines, *, filtered: bool, echo: bool) -> tuple[float, dict]:
    inf = Informer(_LinesClient(lines), R.SECRETS, NS,
                   owner_filter=partition_owner_filter(0, 3) if filtered else None)
    inf.echo_fastpath = True
    inf.add_event_handler(on_add=lambda o: None, on_update=lambda a, b: None)
    await inf._list()
    if echo:  # every line is the echo of a write we published
        for ln in lines:
            o = json.loads(ln)["object"]
            inf.store.assume(o)
    t0 = time.process_time()
    await inf._watch("1")
    dt = time.process_time() - t0
    return dt / len(lines) * 1e6, {"decoded": inf.events - inf.echoes, "echoes": inf.echoes, "filtered": inf.filtered}


async def write_case(n: int, conc: int = 64, server_cpu: dict | None = None) -> float:
    from ncc.kube.kubeconfig import load_kubeconfig, render_kubeconfig
    from ncc.kube.rest import RestClient
    from ncc.shards.shard import slim_written
    from ncc.testing.env import spawn_fakeapi, wait_port_file
    d = tempfile.mkdtemp(prefix="ncc-micro-")
    pf = os.path.join(d, "url")
    proc = spawn_fakeapi("micro", pf)
    try:
        url = wait_port_file(pf, proc)
        kc = os.path.join(d, "kc")
        with open(kc, "w") as f:
            f.write(render_kubeconfig(url, "micro"))
        c = RestClient(load_kubeconfig(kc))
        objs = [make_secret(f"w-{i:05d}", NS, payload=512, version=1) for i in range(conc)]
        rvs = {}
        for o in objs:
            r = await c.create(R.SECRETS, NS, o)
            rvs[o["metadata"]["name"]] = r["metadata"]["resourceVersion"]
        per = n // conc

        async def worker(o):
            nm = o["metadata"]["name"]
            for v in range(per):
                body = dict(o, data={"version": f"{v}".encode().hex()},
                            metadata=dict(o["metadata"], resourceVersion=rvs[nm]))
                _, _, rv, uid = await c.write_meta("update", R.SECRETS, NS, body, name=nm,
                                                   field_manager="nexus-configuration-controller")
                slim_written(R.SECRETS, body, rv, uid)
                rvs[nm] = rv
        import psutil
        sp = psutil.Process(proc.pid)
        s0 = sum(sp.cpu_times()[:2])
        t0 = time.process_time()
        await asyncio.gather(*(worker(o) for o in objs))
        dt = time.process_time() - t0
        if server_cpu is not None:  # the fake apiserver's CPU per write (the substrate's share)
            server_cpu["us"] = min(server_cpu.get("us", 1e18), (sum(sp.cpu_times()[:2]) - s0) / (per * conc) * 1e6)
        await c.close()
        return dt / (per * conc) * 1e6
    finally:
        proc.terminate()
        proc.wait(timeout=10)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=30000)
    ap.add_argument("--writes", type=int, default=20000)
    ap.add_argument("--repeats", type=int, default=5)
    a = ap.parse_args(argv)
    from ncc import native
    native.load(required=True)
    lines = secret_lines(a.lines)
    mine = [ln for i, ln in enumerate(lines) if key_part(f"template/{NS}/algo-{i:05d}", 3) == 0]
    foreign = [ln for i, ln in enumerate(lines) if key_part(f"template/{NS}/algo-{i:05d}", 3) != 0]
    res = {}
    cases = {
        "line_filtered_out_us": lambda: informer_case(foreign, filtered=True, echo=False),
        "line_decoded_us": lambda: informer_case(mine, filtered=True, echo=False),
        "line_decoded_nofilter_us": lambda: informer_case(lines, filtered=False, echo=False),
        "line_echo_confirmed_us": lambda: informer_case(mine, filtered=True, echo=True),
    }
    for name, fn in cases.items():
        best = None
        for _ in range(a.repeats):
            us, counts = asyncio.run(fn())
            best = us if best is None else min(best, us)
        res[name] = round(best, 2)
        res[name.replace("_us", "_counts")] = counts
    srv: dict = {}
    res["write_put_us"] = round(min(asyncio.run(write_case(a.writes, server_cpu=srv))
                                    for _ in range(max(1, a.repeats // 2))), 2)
    res["fakeapi_put_us"] = round(srv.get("us", 0.0), 2)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
