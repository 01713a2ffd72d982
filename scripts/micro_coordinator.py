#!/usr/bin/env python
"""CPU cost of the coordinator's steady-state work per template and wave, without apiservers or executors.

The box's CPUs change speed from run to run (the same tree measures 16k-37k objects/s there), so controller
CPU per object from bench.py cannot resolve a 10 % change.  This drives the coordinator's own code in one
process, with the inputs a bench wave gives it, and times it with `time.process_time`:

* the controller cluster's watch lines of a wave — per template its Secret, its ConfigMap (payload-only
  changes) and the template (new spec, new generation) — through the informers' raw-line path
  (`Informer._consume`: native slim decode of templates, metadata-only skipping of dependents) and the
  watch relay's tap (to one executor);
* one executor report per template (`{"t": "report", ..., "w": true}`) as raw IPC frames through the native
  report table (`Controller.on_executor_stream`);
* the inline finish of every completed key (`finish_inline`) and the Synced Event it records, through the
  broadcaster's correlator and writer tasks to a client that answers at once.

Not included: HTTP (watch chunk parsing, the Event requests and their responses) and the event loop's
socket wake-ups.  Reports µs per template-wave and per object (3 objects per template).

    python scripts/micro_coordinator.py [--templates 1000] [--waves 8] [--profile out.prof]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import struct
import sys
import time

import msgpack

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ncc import native  # noqa: E402
from ncc.api import constants as C  # noqa: E402
from ncc.api import resources as R  # noqa: E402
from ncc.api.refs import ready_condition  # noqa: E402
from ncc.app import strip_payload  # noqa: E402
from ncc.cache.informer import Informer  # noqa: E402
from ncc.controller.controller import Controller  # noqa: E402
from ncc.controller.events import BroadcastRecorder  # noqa: E402
from ncc.controller.options import ControllerOptions  # noqa: E402
from ncc.controller.relay import KINDS, WatchRelay  # noqa: E402
from ncc.testing.workload import configmap_name, make_configmap, make_secret, make_template, secret_name  # noqa: E402

NS = "nexus"
SHARD = "shard-0"


class InstantClient:
    """Answers every write at once (write_meta: the undecoded write the recorder uses)."""
    cluster_name = "controller"

    def __init__(self):
        self.writes = 0

    async def write_meta(self, verb, rt, namespace, body, *, name=None, field_manager=None, patch_type=None,
                         force=None):
        self.writes += 1
        return namespace, name or "", "1", "u"

    async def watch_raw(self, *a, **kw):  # presence selects the informers' raw-line path
        raise NotImplementedError

    async def close(self):
        pass


class _Chan:
    def __init__(self):
        self.sent = 0

    def send_packed(self, b):
        self.sent += 1

    def send(self, m):
        self.sent += 1


class _Handle:
    part, parts = 0, 1

    def __init__(self):
        self.channel = _Chan()


def build(n: int):
    mod = native.load(required=True)
    opts = ControllerOptions.native(native_queue=True, role="coordinator", coalesce_window=0.0)
    client = InstantClient()
    infs = {rt: Informer(client, rt, NS) for rt in (R.TEMPLATES, R.WORKGROUPS, R.SECRETS, R.CONFIGMAPS)}
    for rt in (R.SECRETS, R.CONFIGMAPS):
        infs[rt].metadata_only = True
        infs[rt].store.transform = strip_payload
    infs[R.TEMPLATES].slim_decode = mod.template_event_slim
    recorder = BroadcastRecorder(client, log_events=False, writers=4, coalesce=True, repeat_window=1.0)
    ctl = Controller(alias="controller-cluster", namespace=NS, client=client, shards=[],
                     template_informer=infs[R.TEMPLATES], workgroup_informer=infs[R.WORKGROUPS],
                     secret_informer=infs[R.SECRETS], configmap_informer=infs[R.CONFIGMAPS], options=opts,
                     recorder=recorder, shard_names=[SHARD])
    relay = WatchRelay([infs[rt] for rt in KINDS], infs[R.TEMPLATES].store, NS)
    relay.attach(_Handle())
    state = {"rv": 1}
    objs = {}
    for i in range(n):
        t = make_template(i, NS, secrets=[secret_name(i)], configmaps=[configmap_name(i)])
        name = t["metadata"]["name"]
        uid = f"uid-{name}"
        owner = [{"apiVersion": C.API_VERSION, "kind": C.TEMPLATE_KIND, "name": name, "uid": uid}]
        s = make_secret(secret_name(i), NS)
        c = make_configmap(configmap_name(i), NS)
        for o in (s, c):
            o["metadata"]["ownerReferences"] = owner
            o["metadata"]["uid"] = f"uid-{o['metadata']['name']}"
        t["metadata"].update(uid=uid, generation=1)
        t["status"] = {"conditions": [ready_condition("2026-01-01T00:00:00Z", C.CONDITION_TRUE,
                                                      f"Algorithm {C.go_quote(name)} ready")],
                       "syncedSecrets": [secret_name(i)], "syncedConfigurations": [configmap_name(i)],
                       "syncedToClusters": [SHARD]}
        objs[i] = (s, c, t)
    return ctl, infs, relay, client, objs, state


def line(t: str, obj: dict) -> bytes:
    return json.dumps({"type": t, "object": obj}, separators=(",", ":")).encode()


def wave_lines(objs: dict, state: dict, version: int) -> dict:
    """Per kind, the raw watch lines of one wave, in slices of 100 objects (as the bench's apiserver commits)."""
    out = {R.SECRETS: [], R.CONFIGMAPS: [], R.TEMPLATES: []}
    for i, (s, c, t) in objs.items():
        for rt, o in ((R.SECRETS, s), (R.CONFIGMAPS, c), (R.TEMPLATES, t)):
            state["rv"] += 1
            o["metadata"]["resourceVersion"] = str(state["rv"])
            if rt is R.TEMPLATES:
                o["spec"]["container"]["versionTag"] = f"v{version}"
                o["metadata"]["generation"] = version
            else:
                o["data"]["version"] = str(version)
            out[rt].append(line("ADDED" if version == 1 else "MODIFIED", o))
    return out


def report_frames(objs: dict, version: int) -> bytes:
    buf = bytearray()
    for i, (_s, _c, t) in objs.items():
        body = msgpack.packb({"t": "report", "k": f"template/{NS}/{t['metadata']['name']}", "u": t["metadata"]["uid"],
                              "g": version, "r": {SHARD: None}, "w": True}, use_bin_type=True)
        buf += struct.pack(">I", len(body)) + body
    return bytes(buf)


async def feed(infs, relay, lines: dict, slice_: int = 100) -> None:
    ctxs = {rt: infs[rt]._line_ctx(force=True) for rt in lines}
    n = len(lines[R.TEMPLATES])
    for lo in range(0, n, slice_):
        for rt in (R.SECRETS, R.CONFIGMAPS, R.TEMPLATES):
            batch = lines[rt][lo:lo + slice_]
            relay.on_lines(KINDS.index(rt), batch)
            await infs[rt]._consume(batch, ctxs[rt], "")


async def drain(recorder) -> None:
    while any(q.qsize() for q in recorder._queues) or any(q._unfinished_tasks for q in recorder._queues):
        await asyncio.sleep(0)


async def run(n: int, waves: int, profile: str | None) -> dict:
    ctl, infs, relay, client, objs, state = build(n)
    ctl.recorder.start()
    # cold: list every object into the caches, mark every template adopted at its version, workers "running"
    cold = wave_lines(objs, state, 1)
    await feed(infs, relay, cold)
    for inf in infs.values():
        inf._synced.set()
    for (_s, _c, t) in objs.values():  # adopted at the listed version; the update handler carries the mark
        ctl._adopted[f"template/{NS}/{t['metadata']['name']}"] = t["metadata"]["resourceVersion"]
    ctl.queue.shutdown()  # the cold listing's passes are not part of a wave
    from ncc.workqueue.queue import WorkQueue
    ctl.queue = WorkQueue(native=True)
    ctl.ready.set()
    prepared = [(wave_lines(objs, state, v), report_frames(objs, v)) for v in range(2, waves + 2)]
    prof = None
    if profile:
        import cProfile
        prof = cProfile.Profile()
    times = []
    events0 = ctl.recorder.stats["recorded"]
    for v, (lines, frames) in enumerate(prepared, start=2):
        if prof:
            prof.enable()
        t0 = time.process_time()
        await feed(infs, relay, lines)
        ctl.on_executor_stream(0, frames, 0)
        if ctl._inline_timer is not None:
            ctl._inline_timer.cancel()
        ctl._flush_inline()
        await drain(ctl.recorder)
        dt = time.process_time() - t0
        if prof:
            prof.disable()
        times.append(dt)
    events = ctl.recorder.stats["recorded"] - events0
    await ctl.recorder.stop()
    if prof:
        prof.dump_stats(profile)
    best = min(times)
    return {"templates": n, "waves": waves, "us_per_template_wave": round(best / n * 1e6, 2),
            "us_per_object": round(best / n / 3 * 1e6, 2), "median_us_per_object": round(sorted(times)[len(times) // 2] / n / 3 * 1e6, 2),
            "inline_finishes": ctl.stats["inline_finishes"], "early_passes_skipped": ctl.stats["early_passes_skipped"],
            "events": events, "queued_passes": len(ctl.queue) + ctl.queue.core.waiting()}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--templates", type=int, default=1000)
    ap.add_argument("--waves", type=int, default=8)
    ap.add_argument("--profile", default=None)
    a = ap.parse_args(argv)
    print(json.dumps(asyncio.run(run(a.templates, a.waves, a.profile))))
    return 0


if __name__ == "__main__":
    sys.exit(main())
