"""Resource-type registry: the (group, version, plural, kind) tuples the controller touches.

The reference reaches these through generated typed clients (client-go CoreV1 and the
nexus-core ScienceV1 clientset, main.go:58-68).  Here one generic REST client serves every
type, so a `ResourceType` value carries everything needed to build a URL and to tag an
object with its apiVersion/kind.
"""
from __future__ import annotations

from dataclasses import dataclass

from . import constants as C


@dataclass(frozen=True)
class ResourceType:
    group: str  # "" for the core group
    version: str
    plural: str
    kind: str
    namespaced: bool = True
    has_status: bool = False  # status subresource enabled

    @property
    def api_version(self) -> str:
        return f"{self.group}/{self.version}" if self.group else self.version

    @property
    def list_kind(self) -> str:
        return self.kind + "List"

    @property
    def group_key(self) -> str:
        """Key for per-API-group client state (rate limiters), like client-go's per-group RESTClient."""
        return self.group or "core"

    def base_path(self, namespace: str | None) -> str:
        root = f"/apis/{self.group}/{self.version}" if self.group else f"/api/{self.version}"
        if self.namespaced and namespace:
            return f"{root}/namespaces/{namespace}/{self.plural}"
        return f"{root}/{self.plural}"

    def item_path(self, namespace: str | None, name: str, subresource: str | None = None) -> str:
        p = f"{self.base_path(namespace)}/{name}"
        return f"{p}/{subresource}" if subresource else p

    def __str__(self) -> str:  # pragma: no cover - debugging aid
        return f"{self.plural}.{self.group_key}/{self.version}"


SECRETS = ResourceType("", "v1", "secrets", "Secret")
CONFIGMAPS = ResourceType("", "v1", "configmaps", "ConfigMap")
EVENTS = ResourceType("", "v1", "events", "Event")
NAMESPACES = ResourceType("", "v1", "namespaces", "Namespace", namespaced=False)
TEMPLATES = ResourceType(C.GROUP, C.VERSION, C.TEMPLATE_PLURAL, C.TEMPLATE_KIND, has_status=True)
WORKGROUPS = ResourceType(C.GROUP, C.VERSION, C.WORKGROUP_PLURAL, C.WORKGROUP_KIND, has_status=True)
LEASES = ResourceType("coordination.k8s.io", "v1", "leases", "Lease")  # leader election (ncc/leader.py)

BUILTIN = (SECRETS, CONFIGMAPS, EVENTS, NAMESPACES, TEMPLATES, WORKGROUPS, LEASES)

_BY_KIND = {r.kind: r for r in BUILTIN}
_BY_PLURAL = {(r.group, r.plural): r for r in BUILTIN}


def by_kind(kind: str) -> ResourceType:
    return _BY_KIND[kind]


def by_plural(group: str, plural: str) -> ResourceType | None:
    return _BY_PLURAL.get((group, plural))


def register(rt: ResourceType) -> None:
    """Register an extra resource type (e.g. from a CRD manifest)."""
    _BY_KIND.setdefault(rt.kind, rt)
    _BY_PLURAL[(rt.group, rt.plural)] = rt
