"""Helpers over JSON-shaped Kubernetes objects.

Objects are plain `dict`s exactly as the apiserver serialises them.  The CRD spec is kept
opaque (copied and compared verbatim), which keeps the controller forward compatible with
whatever fields nexus-core adds — SURVEY.md §7.5 mitigation for the absent nexus-core module.

Cached objects are treated as immutable: code that needs a modified object builds a new one
with `with_fields` / `with_meta` (shallow copy-on-write) instead of deep-copying, which is the
hot-path equivalent of client-go's "NEVER modify objects from the store" rule
(controller.go:429-430).
"""
from __future__ import annotations

import time as _time
from typing import Any, NamedTuple

Obj = dict


class ObjectKey(NamedTuple):
    namespace: str
    name: str

    def __str__(self) -> str:
        return f"{self.namespace}/{self.name}" if self.namespace else self.name


def meta(obj: Obj) -> dict:
    m = obj.get("metadata")
    return m if m is not None else {}


def name(obj: Obj) -> str:
    return meta(obj).get("name", "")


def namespace(obj: Obj) -> str:
    return meta(obj).get("namespace", "") or ""


def uid(obj: Obj) -> str:
    return meta(obj).get("uid", "") or ""


def resource_version(obj: Obj) -> str:
    return meta(obj).get("resourceVersion", "") or ""


def labels(obj: Obj) -> dict:
    return meta(obj).get("labels") or {}


def owner_references(obj: Obj) -> list:
    return meta(obj).get("ownerReferences") or []


def key_of(obj: Obj, _new=tuple.__new__, _key=ObjectKey) -> ObjectKey:
    # tuple.__new__ straight away: the NamedTuple's generated __new__ is a Python frame (a third of the cost),
    # and every store upsert and delete computes a key
    m = obj.get("metadata")
    if m is None:
        m = {}
    return _new(_key, (m.get("namespace", "") or "", m.get("name", "")))


def rv_int(rv: str) -> int:
    """Integer view of a resourceVersion (client-go's IntegerResourceVersionMutationCache assumption)."""
    try:
        return int(rv)
    except (TypeError, ValueError):
        return -1


def deep_copy(o: Any) -> Any:
    """Fast deep copy for JSON-shaped data (dict/list/scalars) — ~3x cheaper than copy.deepcopy."""
    t = type(o)
    if t is dict:
        return {k: deep_copy(v) for k, v in o.items()}
    if t is list:
        return [deep_copy(v) for v in o]
    return o


def with_fields(obj: Obj, **fields: Any) -> Obj:
    """Shallow copy of `obj` with top-level fields replaced (copy-on-write)."""
    out = dict(obj)
    out.update(fields)
    return out


def with_meta(obj: Obj, **fields: Any) -> Obj:
    """Shallow copy of `obj` with metadata fields replaced."""
    out = dict(obj)
    m = dict(meta(obj))
    m.update(fields)
    out["metadata"] = m
    return out


_TS_CACHE = [-1, ""]


def now_rfc3339() -> str:
    """metav1.Now() serialised: RFC3339 with second precision, UTC (formatted once per second)."""
    sec = int(_time.time())
    if sec != _TS_CACHE[0]:
        _TS_CACHE[1] = _time.strftime("%Y-%m-%dT%H:%M:%SZ", _time.gmtime(sec))
        _TS_CACHE[0] = sec
    return _TS_CACHE[1]


def normalize_data(d: Any) -> dict:
    """Map a possibly-absent `data` field to a dict (Go nil map == empty map for our purposes)."""
    return d if d else {}
