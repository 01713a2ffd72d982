"""Structural-schema validation of custom resources against their CRD's `openAPIV3Schema`.

A real kube-apiserver validates every write of a custom resource against the CRD's structural
schema and answers 422 Invalid on a type error; the fake apiserver can do the same
(`FakeApiServer(validate_crds=...)`, `python -m ncc.fakeapi --crd-dir`), so the controller's
status and spec writes are held to the contract of the CRDs it ships (deploy/crds, the
reference's nexus-crd chart).  Supported subset (what the NexusAlgorithmTemplate/Workgroup
schemas use): `type` (object, array, string, integer, number, boolean), `properties`, `items`,
`additionalProperties` (schema or bool), `required`, `enum`, `nullable`, `format: int32/int64`
ranges, and `x-kubernetes-preserve-unknown-fields`.  Unknown fields of a non-preserving object
are reported, which on a real apiserver would be pruned (or rejected with strict field validation).
"""
from __future__ import annotations

import copy
import os

import yaml

_INT_RANGES = {"int32": (-2**31, 2**31 - 1), "int64": (-2**63, 2**63 - 1)}


def _type_ok(t: str, v) -> bool:
    if t == "object":
        return isinstance(v, dict)
    if t == "array":
        return isinstance(v, list)
    if t == "string":
        return isinstance(v, str)
    if t == "boolean":
        return isinstance(v, bool)
    if t == "integer":
        return isinstance(v, int) and not isinstance(v, bool)
    if t == "number":
        return isinstance(v, (int, float)) and not isinstance(v, bool)
    return True


def validate(schema: dict, value, path: str = "") -> list[str]:
    """Errors (field path: message) of `value` against a structural schema; [] when valid."""
    errs: list[str] = []
    _walk(schema or {}, value, path, errs)
    return errs


def _walk(s: dict, v, path: str, errs: list) -> None:
    where = path or "<root>"
    if v is None:
        if not s.get("nullable") and s.get("type"):
            errs.append(f"{where}: Invalid value: null: must be {s['type']}")
        return
    t = s.get("type")
    if t and not _type_ok(t, v):
        errs.append(f"{where}: Invalid value: {type(v).__name__}: must be of type {t}")
        return
    if "enum" in s and v not in s["enum"]:
        errs.append(f"{where}: Unsupported value: {v!r}: supported values: {s['enum']}")
    fmt = s.get("format")
    if t == "integer" and fmt in _INT_RANGES:
        lo, hi = _INT_RANGES[fmt]
        if not lo <= v <= hi:
            errs.append(f"{where}: Invalid value: {v}: out of range for {fmt}")
    if isinstance(v, dict):
        props = s.get("properties") or {}
        for r in s.get("required") or ():
            if r not in v:
                errs.append(f"{path + '.' if path else ''}{r}: Required value")
        addl = s.get("additionalProperties")
        preserve = s.get("x-kubernetes-preserve-unknown-fields", False)
        for k, sub in v.items():
            p = f"{path}.{k}" if path else k
            if k in props:
                _walk(props[k], sub, p, errs)
            elif isinstance(addl, dict):
                _walk(addl, sub, p, errs)
            elif addl is True or preserve or (not props and addl is None and not t):
                continue
            elif props or addl is False or t == "object":
                errs.append(f"{p}: Unknown field")
    elif isinstance(v, list) and isinstance(s.get("items"), dict):
        for i, item in enumerate(v):
            _walk(s["items"], item, f"{path}[{i}]", errs)


def default_and_prune(s: dict, v):
    """Apply a structural schema's `default`s to missing properties and drop unknown fields of
    non-preserving objects, in place — what a kube-apiserver does to every custom-resource body it
    decodes (before validation).  Returns `v`."""
    if isinstance(v, dict):
        props = s.get("properties") or {}
        addl = s.get("additionalProperties")
        keep_unknown = addl is True or s.get("x-kubernetes-preserve-unknown-fields", False) or \
            (not props and addl is None and not s.get("type"))
        for k in list(v):
            if k in props:
                default_and_prune(props[k], v[k])
            elif isinstance(addl, dict):
                default_and_prune(addl, v[k])
            elif not keep_unknown:
                del v[k]
        for k, sub in props.items():
            if k not in v and "default" in sub:
                v[k] = copy.deepcopy(sub["default"])
                default_and_prune(sub, v[k])
    elif isinstance(v, list) and isinstance(s.get("items"), dict):
        for item in v:
            default_and_prune(s["items"], item)
    return v


def version_schema(crd: dict, version: str | None = None) -> dict | None:
    vers = (crd.get("spec") or {}).get("versions") or []
    v = next((x for x in vers if version is None or x.get("name") == version), None)
    if v is None:
        return None
    return ((v.get("schema") or {}).get("openAPIV3Schema")) or {}


def default_and_prune_object(crd: dict, obj: dict, version: str | None = None) -> dict:
    """default_and_prune of a custom resource's top-level fields but metadata/apiVersion/kind, in place."""
    schema = version_schema(crd, version)
    if schema is None:
        return obj
    props = schema.get("properties") or {}
    for k in list(obj):
        if k in ("metadata", "apiVersion", "kind"):
            continue
        if k in props:
            default_and_prune(props[k], obj[k])
        elif not schema.get("x-kubernetes-preserve-unknown-fields", False):
            del obj[k]
    for k, sub in props.items():
        if k not in obj and "default" in sub:
            obj[k] = default_and_prune(sub, copy.deepcopy(sub["default"]))
    return obj


def validate_object(crd: dict, obj: dict, version: str | None = None) -> list[str]:
    """Validate a custom resource (spec, status and any other top-level field but metadata/apiVersion/kind)
    against the CRD version's openAPIV3Schema."""
    vers = (crd.get("spec") or {}).get("versions") or []
    v = next((x for x in vers if version is None or x.get("name") == version), None)
    if v is None:
        return [f"version {version} not defined by the CRD"]
    schema = ((v.get("schema") or {}).get("openAPIV3Schema")) or {}
    body = {k: val for k, val in obj.items() if k not in ("metadata", "apiVersion", "kind")}
    return validate(schema, body)


def load_crds(directory: str) -> dict[tuple[str, str], dict]:
    """{(group, plural): CRD document} for every CustomResourceDefinition YAML in `directory`."""
    out = {}
    for fn in sorted(os.listdir(directory)):
        if not fn.endswith((".yaml", ".yml")):
            continue
        with open(os.path.join(directory, fn)) as f:
            for doc in yaml.safe_load_all(f):
                if isinstance(doc, dict) and doc.get("kind") == "CustomResourceDefinition":
                    spec = doc.get("spec") or {}
                    out[(spec.get("group", ""), (spec.get("names") or {}).get("plural", ""))] = doc
    return out
