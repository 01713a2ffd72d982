"""Template reference extraction, owner references and status conditions.

Re-creates the parts of the nexus-core `science/v1` API the controller relies on
(SURVEY.md §2.2, X1a/X1b/X8g):

* `secret_names` / `configmap_names` — `NexusAlgorithmTemplate.GetSecretNames()` /
  `GetConfigMapNames()`: names from `spec.runtimeEnvironment.mappedEnvironmentVariables[*]`
  `.secretRef.name` / `.configMapRef.name`, skipping entries without that ref
  (controller_test.go:261-282 builds zero-valued EnvFromSource entries when refs are nil).
* `template_owner_ref` — the owner reference appended by adoption and by shard-side creates,
  with no `controller`/`blockOwnerDeletion` (controller.go:656-661, controller_test.go:203-208).
* `ready_condition` — `v1.NewResourceReadyCondition(time, status, message)`.
"""
from __future__ import annotations

from . import constants as C
from .objects import Obj, meta


def _mapped_env(template: Obj) -> list:
    spec = template.get("spec") or {}
    rt = spec.get("runtimeEnvironment") or {}
    return rt.get("mappedEnvironmentVariables") or []


def secret_names(template: Obj, unique: bool = False) -> list[str]:
    out: list[str] = []
    for ef in _mapped_env(template):
        ref = (ef or {}).get("secretRef")
        if ref is not None:
            out.append(ref.get("name", ""))
    return _dedupe(out) if unique else out


def configmap_names(template: Obj, unique: bool = False) -> list[str]:
    out: list[str] = []
    for ef in _mapped_env(template):
        ref = (ef or {}).get("configMapRef")
        if ref is not None:
            out.append(ref.get("name", ""))
    return _dedupe(out) if unique else out


def dependent_names(template: Obj) -> tuple[list[str], list[str]]:
    """(`secret_names`, `configmap_names`) in one walk over the mapped environment."""
    secrets: list[str] = []
    configmaps: list[str] = []
    for ef in _mapped_env(template):
        if ef:
            ref = ef.get("secretRef")
            if ref is not None:
                secrets.append(ref.get("name", ""))
            ref = ef.get("configMapRef")
            if ref is not None:
                configmaps.append(ref.get("name", ""))
    return secrets, configmaps


def same_references(old: Obj, new: Obj) -> bool:
    """True when two template versions reference the same Secrets and ConfigMaps (in order).  Identical
    mapped-environment lists, the common case of a version bump, are recognised by one C-level compare."""
    sa, sb = old.get("spec"), new.get("spec")
    if sa and sb:
        ra = sa.get("_rfp")  # slim templates (_native.template_event_slim): a digest of the references' text
        if ra is not None and ra == sb.get("_rfp"):
            return True
    a, b = _mapped_env(old), _mapped_env(new)
    return a == b or dependent_names(old) == dependent_names(new)


def _dedupe(xs: list[str]) -> list[str]:
    seen: set[str] = set()
    out = []
    for x in xs:
        if x not in seen:
            seen.add(x)
            out.append(x)
    return out


def template_owner_ref(template: Obj) -> dict:
    m = meta(template)
    return {
        "apiVersion": C.API_VERSION,
        "kind": C.TEMPLATE_KIND,
        "name": m.get("name", ""),
        "uid": m.get("uid", "") or "",
    }


def is_owned_by_uid(obj: Obj, owner_uid: str) -> bool:
    """controller.go:637-645 — any ownerRef carrying the template UID (kind not checked)."""
    for ref in meta(obj).get("ownerReferences") or ():
        if (ref.get("uid", "") or "") == owner_uid:
            return True
    return False


def template_owner_names(obj: Obj) -> list[str]:
    """Names of NexusAlgorithmTemplate owners of a dependent (controller.go:208-222)."""
    return [r.get("name", "") for r in meta(obj).get("ownerReferences") or () if r.get("kind") == C.TEMPLATE_KIND]


def ready_condition(last_transition_time: str, status: str, message: str) -> dict:
    return {
        "type": C.CONDITION_READY,
        "status": status,
        "lastTransitionTime": last_transition_time,
        "reason": C.CONDITION_READY_REASON,
        "message": message,
    }
