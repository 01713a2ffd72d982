"""Shard discovery from a directory of kubeconfig files (nexus-core `shards.LoadShards`).

Every `*.kubeconfig` file in `shard_config_path` is one shard; the shard name is the file name
without the suffix (CI: `kind-nexus-shard-0.kubeconfig`, controller_test.go:1289).  The Helm
chart mounts the `shardsConfigSecretName` Secret there, one data key per shard
(README.md:15-28, .helm/templates/deployment.yaml:106-124).  Shards are returned in file-name
order — the order the reference iterates them (controller.go:790) — with their informers
started, since `main()` never starts shard factories itself (main.go:73).
"""
from __future__ import annotations

import logging
import os
from typing import Callable

from ..api import resources as R
from ..kube.client import KubeClient, RateLimitedClient
from ..kube.kubeconfig import load_kubeconfig
from ..kube.rest import RestClient
from .shard import Shard

log = logging.getLogger("ncc.shards")

SUFFIX = ".kubeconfig"


def discover(shard_config_path: str) -> list[tuple[str, str]]:
    """[(shard name, kubeconfig path)] sorted by name; Kubernetes secret-volume `..data` symlinks skipped."""
    if not shard_config_path or not os.path.isdir(shard_config_path):
        return []
    out = []
    for fn in sorted(os.listdir(shard_config_path)):
        if fn.startswith(".") or not fn.endswith(SUFFIX):
            continue
        p = os.path.join(shard_config_path, fn)
        if os.path.isfile(p):
            out.append((fn[: -len(SUFFIX)], p))
    return out


def default_client_factory(qps: float = 0.0, burst: int = 10, pool_size: int = 64,
                           transport: str = "fast", pipeline_depth: int = 1,
                           http2: str = "auto") -> Callable[[str, str], KubeClient]:
    def make(name: str, path: str) -> KubeClient:
        client: KubeClient = RestClient(load_kubeconfig(path, name=name), pool_size=pool_size, cluster_name=name,
                                        transport=transport, pipeline_depth=pipeline_depth, http2=http2)
        if qps > 0:
            client = RateLimitedClient(client, qps, burst)
        return client
    return make


def load_shards(alias: str, shard_config_path: str, namespace: str, *,
                client_factory: Callable[[str, str], KubeClient] | None = None, resync_period: float = 0.0,
                assume_writes: bool = False, sync_binary_data: bool = False, sync_metadata: bool = False,
                slim: bool = False,
                start: bool = True, names: set | None = None, key_filter=None, owner_filter=None) -> list[Shard]:
    from ..controller.reconcile import slim_data, slim_spec
    make = client_factory or default_client_factory()
    transforms = {R.TEMPLATES: slim_spec, R.WORKGROUPS: slim_spec, R.SECRETS: slim_data,
                  R.CONFIGMAPS: slim_data} if slim else None
    shards = []
    for name, path in discover(shard_config_path):
        if names is not None and name not in names:
            continue
        client = make(name, path)
        shard = Shard(alias, name, client, namespace, resync_period=resync_period, assume_writes=assume_writes,
                      sync_binary_data=sync_binary_data, sync_metadata=sync_metadata, transforms=transforms,
                      key_filters={R.TEMPLATES: key_filter, R.WORKGROUPS: key_filter} if key_filter else None,
                      owner_filters={R.SECRETS: owner_filter, R.CONFIGMAPS: owner_filter} if owner_filter else None)
        if start:
            shard.start()
        shards.append(shard)
        log.info("loaded shard %s from %s", name, path)
    return shards
