"""Randomised chaos against the native topology, checked against a model of the end state.

A seeded sequence of user changes — template spec updates, Secret/ConfigMap payload updates, new templates
(some sharing an existing dependent), templates pointed at another Secret, a referenced ConfigMap deleted
and re-created, template deletes — runs while the shards misbehave: a share of their
writes fail (503), a shard apiserver goes down and comes back, watch streams are cut, the watch history is
compacted (resumes get 410 and relist), and executor processes are killed (the pool respawns them with a fresh snapshot).  Once the faults clear,
every shard must hold exactly what the controller cluster implies:

* every controller template, with the same spec, Ready with every shard listed;
* every dependent a template references, with the controller's payload and an ownerRef to the shard copy
  of each template that references it;
* no copy of a deleted template (queued, retried deletes), and no dependent that only it owned (shard GC).

Runs for the in-process topology and for the Python and C++ executors (executor kills only where there
are executors).  NCC_CHAOS_STEPS / NCC_CHAOS_SEEDS / NCC_CHAOS_KILLS scale a run up for exploration.
"""
import asyncio
import os
import random

import pytest

from ncc.api import constants as C
from ncc.api import resources as R
from ncc.testing.workload import make_configmap, make_secret, make_template

from test_conformance import NS, Cluster, mutate, wait_for

pytestmark = pytest.mark.skipif(os.environ.get("NCC_SKIP_CHAOS") == "1", reason="NCC_SKIP_CHAOS=1")
# NCC_CHAOS_STEPS / NCC_CHAOS_SEEDS / NCC_CHAOS_KILLS scale the run up for exploration
STEPS = int(os.environ.get("NCC_CHAOS_STEPS", "40"))
SEEDS = int(os.environ.get("NCC_CHAOS_SEEDS", "5"))
MAX_KILLS = int(os.environ.get("NCC_CHAOS_KILLS", "2"))


def _deps(t: dict) -> tuple[list, list]:
    mev = t["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"]
    return ([e["secretRef"]["name"] for e in mev if e.get("secretRef")],
            [e["configMapRef"]["name"] for e in mev if e.get("configMapRef")])


def _missing_refs(cl, t) -> list:
    """The Secrets / ConfigMaps template `t` references that do not exist on the controller cluster."""
    if t is None:
        return []
    secrets, cms = _deps(t)
    return [n for n in secrets if cl.cstate.try_get(R.SECRETS, NS, n) is None] + \
        [n for n in cms if cl.cstate.try_get(R.CONFIGMAPS, NS, n) is None]


def _converged(cl, active=None, meta_sync: bool = False) -> str:
    """'' when every (active) shard matches the model, else the first difference found."""
    active = sorted(active if active is not None else range(len(cl.sstates)))
    shards = [cl.env.shard_names[i] for i in active]
    templates = {t["metadata"]["name"]: t for t in cl.cstate.list(R.TEMPLATES, NS)["items"]}
    missing_events = None
    for name, t in list(templates.items()):
        missing = _missing_refs(cl, t)
        if missing:
            # a reference that does not exist: the controller-side GC deleted a Secret the user re-pointed this
            # template at while its previous owners went (adoption made it theirs) — the
            # reference fails such a template with ErrResourceMissing until the Secret is back, and so do we:
            # its shard copies are not checked, its Warning Event is
            if missing_events is None:
                missing_events = [e for e in cl.cstate.list(R.EVENTS, NS)["items"]
                                  if e["reason"] == C.ERR_RESOURCE_MISSING]
            for n in missing:
                want = C.MESSAGE_RESOURCE_MISSING.format(f'"{n}"', f'"{name}"')
                if not any(e["involvedObject"]["name"] == name and want in e.get("message", "")
                           for e in missing_events):
                    return f"{name}: no {C.ERR_RESOURCE_MISSING} event for its missing reference {n}"
            templates.pop(name)
    for name, t in templates.items():
        st = t.get("status") or {}
        c = (st.get("conditions") or [{}])[0]
        if c.get("status") != "True" or st.get("syncedToClusters") != shards:
            return f"{name}: status {c.get('status')} {st.get('syncedToClusters')} {c.get('message', '')[:300]!r}"
    for i, s in ((i, cl.sstates[i]) for i in active):
        ours = {t["metadata"]["name"]: t for t in s.list(R.TEMPLATES, NS)["items"]}
        every = {t["metadata"]["name"] for t in cl.cstate.list(R.TEMPLATES, NS)["items"]}
        # a template with a missing reference may or may not have reached this shard before the reference went
        if not set(templates) <= set(ours) <= every:
            return f"shard {i}: templates {sorted((set(templates) - set(ours)) | (set(ours) - every))} differ"
        want_owners: dict = {}
        for name, t in templates.items():
            if ours[name]["spec"] != t["spec"]:
                return f"shard {i}: {name} spec differs"
            secrets, cms = _deps(t)
            for rt, names in ((R.SECRETS, secrets), (R.CONFIGMAPS, cms)):
                for n in names:
                    want_owners.setdefault((rt.plural, n), set()).add(ours[name]["metadata"]["uid"])
        for (plural, n), uids in want_owners.items():
            rt = R.SECRETS if plural == "secrets" else R.CONFIGMAPS
            live = s.try_get(rt, NS, n)
            if live is None:
                return f"shard {i}: {plural}/{n} missing"
            src = cl.cstate.get(rt, NS, n)
            if live.get("data") != src.get("data"):
                return f"shard {i}: {plural}/{n} data differs"
            if meta_sync:  # sync-dependent-metadata: the copy carries the source's labels and annotations
                for mk in ("labels", "annotations"):
                    want, have = src["metadata"].get(mk) or {}, dict(live["metadata"].get(mk) or {})
                    for k in list(C.owner_labels("controller-cluster")) + [C.SYNCED_METADATA_ANNOTATION]:
                        have.pop(k, None)  # ours, not the source's (nothing else writes the copies here)
                    if have != want:
                        return f"shard {i}: {plural}/{n} {mk} {have} != {want}"
            have = {r["uid"] for r in live["metadata"].get("ownerReferences") or ()}
            if not uids <= have:
                return f"shard {i}: {plural}/{n} owners {sorted(have)} lack {sorted(uids - have)}"
        live_uids = {t["metadata"]["uid"] for t in ours.values()}
        for rt in (R.SECRETS, R.CONFIGMAPS):
            for o in s.list(rt, NS)["items"]:
                if (rt.plural, o["metadata"]["name"]) not in want_owners:
                    # no longer referenced: kept while a live template still owns it (the reference never
                    # removes ownerRefs), collected by the shard's GC once all its owners are gone
                    owners = {r["uid"] for r in o["metadata"].get("ownerReferences") or ()}
                    if owners and not owners & live_uids:
                        return f"shard {i}: {rt.plural}/{o['metadata']['name']} left behind by a deleted template"
    return ""


@pytest.mark.parametrize("topology", ["inprocess", "python", "native", "native-c2", "native-reload", "native-ssa",
                                      "native-meta", "native-h2", "python-h2"])
@pytest.mark.parametrize("seed", list(range(1, SEEDS + 1)))
async def test_chaos_converges_to_the_model(tmp_path, topology, seed, monkeypatch):
    """`native-c2`: two coordinator partitions (a child coordinator process owns half the template keys);
    the kills then also hit the child coordinator.  `native-ssa`: shard writes by server-side apply.
    `native-meta`: sync-dependent-metadata, with source labels/annotations changed along the way.
    `native-h2`: the C++ executors write to the shards over HTTP/2 (`client-http2: on`, prior knowledge);
    `python-h2`: the same with the Python executors (ncc/kube/h2client.py on every shard connection)."""
    from ncc.controller.native_executor import binary_path
    reload = topology.endswith("-reload")
    ssa = topology.endswith("-ssa")
    meta_sync = topology.endswith("-meta")
    h2 = topology.endswith("-h2")
    impl, _, parts = topology.replace("-reload", "").replace("-ssa", "").replace("-meta", "").replace(
        "-h2", "").partition("-c")
    if impl == "native" and binary_path() is None:
        pytest.skip("ncc/bin/ncc-executor is not built")
    monkeypatch.delenv("NCC_EXECUTOR_IMPL", raising=False)
    rnd = random.Random(seed)
    extra = {"coordinator_partitions": int(parts)} if parts else {}
    if reload:  # a third shard whose kubeconfig comes and goes (hot reload of the shards directory)
        extra["shard_reload_period"] = 0
    if ssa:
        extra["server_side_apply"] = True
    if meta_sync:
        extra["sync_dependent_metadata"] = True
    if h2:
        extra["client_http2"] = "on"
    if os.environ.get("NCC_CHAOS_LOG"):
        extra["log_level"] = os.environ["NCC_CHAOS_LOG"]
    async with Cluster(tmp_path, impl, n_shards=3 if reload else 2, **extra) as cl:
        active = set(range(len(cl.sstates)))
        if reload:
            kc = os.path.join(cl.env.shard_dir, "shard-2.kubeconfig")
            parked = os.path.join(str(tmp_path), "shard-2.kubeconfig.parked")
            os.replace(kc, parked)
            active = {0, 1}
        live = []
        for i in range(6):
            cl.seed(i, secrets=(f"s{i}",), configmaps=(f"c{i}",))
            live.append(f"algo-{i:05d}")
        await cl.start()
        next_id, kills, version, downs = 6, 0, 0, 0
        ops: dict = {}
        for _step in range(STEPS):
            version += 1
            op = rnd.choices(["spec", "secret", "configmap", "create", "delete", "fault", "kill", "reref",
                              "recreate", "reshard", "relabel"],
                             weights=[5, 4, 3, 2, 2, 3, 1, 2, 1, 2 if reload else 0, 3 if meta_sync else 0])[0]
            ops[op] = ops.get(op, 0) + 1
            if op == "spec" and live:
                name = rnd.choice(live)
                await mutate(cl.cc, R.TEMPLATES, name,
                             lambda o, v=version: o["spec"]["container"].__setitem__("versionTag", f"v{v}"))
            elif op in ("secret", "configmap"):
                rt = R.SECRETS if op == "secret" else R.CONFIGMAPS
                names = [o["metadata"]["name"] for o in cl.cstate.list(rt, NS)["items"]]
                if names:
                    n = rnd.choice(names)
                    val = f"v{version}" if rt is R.CONFIGMAPS else "djk="
                    await mutate(cl.cc, rt, n, lambda o, k=f"k{version}", v=val: o.setdefault("data", {})
                                 .__setitem__(k, v))
            elif op == "create":
                i = next_id
                next_id += 1
                shared = rnd.random() < 0.3 and live
                sec = f"s{rnd.randrange(next_id - 1)}" if shared else f"s{i}"
                if cl.cstate.try_get(R.SECRETS, NS, sec) is None:
                    await cl.cc.create(R.SECRETS, NS, make_secret(sec, NS))
                await cl.cc.create(R.CONFIGMAPS, NS, make_configmap(f"c{i}", NS))
                await cl.cc.create(R.TEMPLATES, NS, make_template(i, NS, secrets=[sec], configmaps=[f"c{i}"]))
                live.append(f"algo-{i:05d}")
            elif op == "reref" and live:
                # point a template at another Secret (an existing one, or a new one)
                name = rnd.choice(live)
                names = [o["metadata"]["name"] for o in cl.cstate.list(R.SECRETS, NS)["items"]]
                target = rnd.choice(names) if names and rnd.random() < 0.5 else f"sx{version}"
                if cl.cstate.try_get(R.SECRETS, NS, target) is None:
                    await cl.cc.create(R.SECRETS, NS, make_secret(target, NS))

                def reref(o, target=target):
                    mev = o["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"]
                    o["spec"]["runtimeEnvironment"]["mappedEnvironmentVariables"] = \
                        [e for e in mev if not e.get("secretRef")] + [{"secretRef": {"name": target}}]
                await mutate(cl.cc, R.TEMPLATES, name, reref)
            elif op == "recreate":
                # a referenced ConfigMap deleted and created again (its references go missing meanwhile)
                names = [o["metadata"]["name"] for o in cl.cstate.list(R.CONFIGMAPS, NS)["items"]]
                if names:
                    n = rnd.choice(names)
                    await cl.cc.delete(R.CONFIGMAPS, NS, n)
                    await asyncio.sleep(rnd.uniform(0, 0.05))
                    await cl.cc.create(R.CONFIGMAPS, NS, make_configmap(n, NS, version=version))
            elif op == "relabel":  # a source's labels/annotations change (a key set, changed or removed)
                rt = rnd.choice([R.SECRETS, R.CONFIGMAPS])
                names = [o["metadata"]["name"] for o in cl.cstate.list(rt, NS)["items"]]
                if names:
                    mk, key = rnd.choice(["labels", "annotations"]), rnd.choice(["team", "tier", "note"])

                    def relabel(o, mk=mk, key=key, v=f"v{version}", drop=rnd.random() < 0.4):
                        d = o["metadata"].setdefault(mk, {}) or {}
                        if drop:
                            d.pop(key, None)
                        else:
                            d[key] = v
                        o["metadata"][mk] = d
                    await mutate(cl.cc, rt, rnd.choice(names), relabel)
            elif op == "reshard":  # shard-2 joins or leaves
                if 2 in active:
                    os.replace(kc, parked)
                    active.discard(2)
                else:
                    os.replace(parked, kc)
                    active.add(2)
                await cl.app.reload_shards()
            elif op == "delete" and len(live) > 2:
                name = live.pop(rnd.randrange(len(live)))
                await cl.cc.delete(R.TEMPLATES, NS, name)
            elif op == "fault":
                srv = rnd.choice(cl.env.shard_servers)
                kind = rnd.choice(["errors", "drop", "compact", "down", "up"])
                if kind == "errors":
                    srv.faults.update({"error_rate": 0.2, "error_code": 503})
                elif kind in ("down", "up"):  # the whole shard apiserver unavailable (503 to everything)
                    srv.faults.update({"down": kind == "down"})
                    if kind == "down":
                        srv.drop_watches()
                        downs += 1
                elif kind == "drop":
                    srv.drop_watches()
                else:
                    srv.state.compact()
                    srv.drop_watches()
            elif op == "kill" and kills < MAX_KILLS and cl.app.pool is not None:
                h = rnd.choice(cl.app.pool.handles + (cl.app.partitions.handles if cl.app.partitions else []))
                if h.proc is not None and h.proc.returncode is None:
                    h.proc.kill()  # a crash: the pool respawns it (not `h.kill()`, which stops it for good)
                    kills += 1
            await asyncio.sleep(rnd.uniform(0, 0.03))
        for srv in cl.env.shard_servers:
            srv.faults.update({"error_rate": 0.0, "down": False})
        print(f"seed {seed} {topology}: ops {ops}, process kills {kills}, templates {len(live)}")
        last = ""

        async def done():
            nonlocal last
            last = _converged(cl, active, meta_sync)
            return last == ""
        streak = [0]

        async def settled():  # converged, and still so a second later: no pass of the chaos phase in flight
            streak[0] = streak[0] + 1 if await done() else 0
            return streak[0] >= 6

        try:
            await wait_for(settled, timeout=45, interval=0.2)
        except AssertionError:
            raise AssertionError(f"seed {seed} ({topology}) did not converge: {last}") from None
        rogue = [e for e in cl.cstate.list(R.EVENTS, NS)["items"] if e["reason"] == C.ERR_RESOURCE_EXISTS]
        assert rogue == []  # nothing here is a rogue object
        # the model check sees a difference (and the controller repairs it): drift on one shard copy.  After
        # a "down" episode too: a shard watch in its reconnect backoff (client-go's 0.8 s doubling to 30 s)
        # retries as soon as the shard answers the executor's writes again.
        # (a template the model checks: not one whose reference the controller-side GC removed — its shard copy
        # is legitimately left alone, see _converged)
        checked = [n for n in live if not _missing_refs(cl, cl.cstate.try_get(R.TEMPLATES, NS, n))]
        name = checked[0] if checked else None
        if name is None:
            return
        drifted = await mutate(cl.sc[0], R.TEMPLATES, name,
                               lambda o: o["spec"]["container"].__setitem__("versionTag", "drift"))
        seen = _converged(cl, active)
        if "spec differs" not in seen:
            # already repaired: the C++ executor can answer the drift's watch event before this client has read
            # the response to its own write — then the copy was written again after the drift
            cur = await cl.sc[0].get(R.TEMPLATES, NS, name)
            assert int(cur["metadata"]["resourceVersion"]) > int(drifted["metadata"]["resourceVersion"]), (seen, cur)
        try:
            await wait_for(done, timeout=15, interval=0.1)
        except AssertionError:
            import json as _json
            st = cl.app.debug_state().get("executors") if cl.app is not None else None
            raise AssertionError(f"seed {seed} ({topology}): drift on shard-0 not repaired: {last}; executors: "
                                 f"{_json.dumps(st, default=str)[:3000]}") from None
