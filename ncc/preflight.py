"""`python -m ncc --check-shards`: a preflight for a deployment (docs/MIGRATION.md, step 2).

Loads the controller cluster's kubeconfig and every `<cluster>.kubeconfig` in `shard-config-path` exactly as
the controller does (credentials, `exec` plugins, CA), then LISTs each kind the controller reads and writes
in `controller-namespace` on each cluster.  One JSON line per cluster, then a summary line; exit status 0 when
every cluster answered every list.  A missing CRD shows up as NotFound, missing RBAC as Forbidden, a wrong
server or CA as TransportError — before the controller starts and waits for caches that never sync.  Each
line also names the protocol negotiated (`h2` or `http/1.1`, per `client-http2`).  Write permissions are not probed (that would need writes, or SelfSubjectAccessReviews the reference never needed).
"""
from __future__ import annotations

import asyncio
import json

from .api import resources as R
from .config import controller_http2
from .kube import errors as E
from .kube.kubeconfig import build_config, load_kubeconfig
from .kube.rest import RestClient
from .shards.loader import discover

KINDS = (R.TEMPLATES, R.WORKGROUPS, R.SECRETS, R.CONFIGMAPS)


async def check_cluster(name: str, client, namespace: str, timeout: float = 10.0) -> dict:
    kinds = {}
    unreachable = False
    for rt in KINDS:
        if unreachable:  # one timeout or connection failure is enough: do not wait again per kind
            kinds[rt.plural] = "skipped (cluster unreachable)"
            continue
        try:
            await asyncio.wait_for(client.list(rt, namespace, limit=1), timeout)
            kinds[rt.plural] = "ok"
        except asyncio.TimeoutError:
            kinds[rt.plural] = f"TransportError: no answer within {timeout:g}s"
            unreachable = True
        except E.TransportError as e:
            kinds[rt.plural] = f"TransportError: {e}"[:300]
            unreachable = True
        except E.ApiError as e:
            kinds[rt.plural] = f"{type(e).__name__} ({e.code}): {e.message}"[:300]
        except Exception as e:  # noqa: BLE001 - TLS and other client-side failures
            kinds[rt.plural] = f"{type(e).__name__}: {e}"[:300]
    out = {"cluster": name, "ok": all(v == "ok" for v in kinds.values()), "kinds": kinds}
    proto = getattr(client, "protocol", None)
    if proto is not None:  # what the controller will speak to it (client-http2: HTTP/2 where TLS negotiates it)
        out["protocol"] = proto
    return out


async def check(cfg, timeout: float = 10.0) -> list[dict]:
    out = []
    targets = [("controller", lambda: build_config(cfg.controller_config_path))]
    targets += [(name, (lambda p=path, n=name: load_kubeconfig(p, name=n)))
                for name, path in discover(cfg.shard_config_path)]
    for name, make_cfg in targets:
        try:
            mode = controller_http2(cfg.client_http2) if name == "controller" else cfg.client_http2
            client = RestClient(make_cfg(), pool_size=2, cluster_name=name, http2=mode)
        except Exception as e:  # noqa: BLE001 - an unreadable kubeconfig
            out.append({"cluster": name, "ok": False, "error": f"{type(e).__name__}: {e}"[:300]})
            continue
        try:
            out.append(await check_cluster(name, client, cfg.controller_namespace, timeout))
        finally:
            await client.close()
    return out


def run(cfg, print_fn=print) -> int:
    results = asyncio.run(check(cfg))
    for r in results:
        print_fn(json.dumps(r, sort_keys=True))
    shards = [r for r in results if r["cluster"] != "controller"]
    ok = all(r["ok"] for r in results) and bool(shards)
    print_fn(json.dumps({"summary": "ok" if ok else "failed", "clusters": len(results), "shards": len(shards),
                         "failing": [r["cluster"] for r in results if not r["ok"]]
                         + ([] if shards else ["(no *.kubeconfig in shard-config-path)"])}))
    return 0 if ok else 1
