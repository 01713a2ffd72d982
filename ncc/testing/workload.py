"""Synthetic Nexus workload: algorithm templates targeting MI355X shard nodes, their Secrets/ConfigMaps, workgroups.

Shapes follow the reference test objects (controller_test.go:230-333) scaled to benchmark
sizes (BASELINE.json configs).  Templates request `amd.com/gpu` in
`computeResources.customResources` and workgroups tolerate the `amd.com/gpu` taint — the
shard clusters these configs land on are 8×MI355X nodes.
"""
from __future__ import annotations

import base64

from ..api import constants as C


def template_name(i: int) -> str:
    return f"algo-{i:05d}"


def secret_name(i: int) -> str:
    return f"algo-{i:05d}-secret"


def configmap_name(i: int) -> str:
    return f"algo-{i:05d}-config"


def make_template(i: int, namespace: str, *, secrets: list[str] = (), configmaps: list[str] = (),
                  version: str = "v1.0.0", gpus: int = 8) -> dict:
    env_from = [{"secretRef": {"name": s}} for s in secrets] + [{"configMapRef": {"name": c}} for c in configmaps]
    return {
        "apiVersion": C.API_VERSION,
        "kind": C.TEMPLATE_KIND,
        "metadata": {"name": template_name(i), "namespace": namespace},
        "spec": {
            "container": {"image": f"algorithms/algo-{i % 97}", "registry": "registry.example.com",
                          "versionTag": version, "serviceAccountName": "nexus-algorithm"},
            "computeResources": {"cpuLimit": "32000m", "memoryLimit": "512Gi",
                                 "customResources": {"amd.com/gpu": str(gpus)}},
            "workgroupRef": {"name": "mi355x", "group": C.GROUP, "kind": C.WORKGROUP_KIND},
            "command": "python",
            "args": ["-m", "algorithm.main", f"--shard-index={i}"],
            "runtimeEnvironment": {
                "environmentVariables": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"},
                                         {"name": "NCCL_MIN_NCHANNELS", "value": "32"}],
                "mappedEnvironmentVariables": env_from,
                "annotations": {"nexus/algorithm-index": str(i)},
                "deadlineSeconds": 3600,
                "maximumRetries": 3,
            },
            "errorHandlingBehaviour": {"transientExitCodes": [137, 143], "fatalExitCodes": [1]},
            "datadogIntegrationSettings": {"mountDatadogSocket": True},
        },
    }


def make_secret(name: str, namespace: str, *, payload: int = 256, version: int = 0) -> dict:
    raw = (f"{name}:{version}:".encode() * (payload // max(len(name), 1) + 1))[:payload]
    return {"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
            "metadata": {"name": name, "namespace": namespace},
            "data": {"token": base64.b64encode(raw).decode(), "version": base64.b64encode(str(version).encode()).decode()}}


def make_configmap(name: str, namespace: str, *, payload: int = 256, version: int = 0) -> dict:
    return {"apiVersion": "v1", "kind": "ConfigMap",
            "metadata": {"name": name, "namespace": namespace},
            "data": {"config.yaml": f"# {name} v{version}\n" + ("x" * payload), "version": str(version)}}


def make_workgroup(name: str, namespace: str, cluster: str = "") -> dict:
    return {
        "apiVersion": C.API_VERSION,
        "kind": C.WORKGROUP_KIND,
        "metadata": {"name": name, "namespace": namespace},
        "spec": {"description": "MI355X training/serving pool", "capabilities": {"gpu": True, "xgmi": True},
                 "cluster": cluster,
                 "tolerations": [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}],
                 "affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                     "nodeSelectorTerms": [{"matchExpressions": [
                         {"key": "node.kubernetes.io/instance-type", "operator": "In",
                          "values": ["mi355x-8gpu"]}]}]}}}},
    }


def template_set(n: int, namespace: str, *, secrets_per: int = 1, configmaps_per: int = 1, version: str = "v1.0.0",
                 payload: int = 256) -> tuple[list, list, list]:
    """(templates, secrets, configmaps) with per-template dependents."""
    ts, ss, cs = [], [], []
    for i in range(n):
        snames = [secret_name(i) if k == 0 else f"{secret_name(i)}-{k}" for k in range(secrets_per)]
        cnames = [configmap_name(i) if k == 0 else f"{configmap_name(i)}-{k}" for k in range(configmaps_per)]
        ts.append(make_template(i, namespace, secrets=snames, configmaps=cnames, version=version))
        ss.extend(make_secret(s, namespace, payload=payload) for s in snames)
        cs.extend(make_configmap(c, namespace, payload=payload) for c in cnames)
    return ts, ss, cs
