"""Patch application used by the fake apiserver (and available to tests).

* RFC 7386 JSON merge patch (`application/merge-patch+json`).  Strategic merge patch is
  approximated by merge patch except that `metadata.ownerReferences` lists are merged by
  `uid`, which is the only strategic list this controller relies on.
* RFC 6902 JSON patch (`add`/`remove`/`replace`/`test`/`copy`/`move`).
* An approximation of server-side apply: fields present in the applied configuration replace the
  live ones; labels/annotations are merged; ownerReferences are unioned by uid.  The fake apiserver's
  storage (`ClusterState.patch`) also tracks what each field manager applied and removes a top-level
  field, label, annotation or ownerReference entry the same manager applied before and omits now
  (an ownerReference another manager also applies stays), as real SSA does from managedFields.
"""
from __future__ import annotations

from .objects import deep_copy


def merge_patch(target, patch):
    if not isinstance(patch, dict):
        return deep_copy(patch)
    out = dict(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def strategic_merge_patch(target: dict, patch: dict) -> dict:
    refs = (patch.get("metadata") or {}).get("ownerReferences") if isinstance(patch, dict) else None
    out = merge_patch(target, patch)
    if refs is not None:
        live = list((target.get("metadata") or {}).get("ownerReferences") or [])
        by_uid = {r.get("uid"): i for i, r in enumerate(live)}
        for r in refs:
            if r.get("uid") in by_uid:
                live[by_uid[r.get("uid")]] = r
            else:
                live.append(r)
        out.setdefault("metadata", {})["ownerReferences"] = live
    return out


def _ptr(path: str) -> list[str]:
    if path == "":
        return []
    if not path.startswith("/"):
        raise ValueError(f"invalid JSON pointer {path!r}")
    return [p.replace("~1", "/").replace("~0", "~") for p in path[1:].split("/")]


def _walk(doc, parts):
    cur = doc
    for p in parts:
        cur = cur[int(p)] if isinstance(cur, list) else cur[p]
    return cur


def json_patch(doc, ops: list) -> dict:
    doc = deep_copy(doc)
    for op in ops:
        kind = op["op"]
        parts = _ptr(op["path"])
        if kind == "test":
            if _walk(doc, parts) != op.get("value"):
                raise ValueError(f"test failed at {op['path']}")
            continue
        if kind in ("copy", "move"):
            src = _ptr(op["from"])
            val = deep_copy(_walk(doc, src))
            if kind == "move":
                parent = _walk(doc, src[:-1])
                if isinstance(parent, list):
                    parent.pop(int(src[-1]))
                else:
                    del parent[src[-1]]
            op = {"op": "add", "path": op["path"], "value": val}
            kind = "add"
        if not parts:
            if kind in ("add", "replace"):
                doc = deep_copy(op["value"])
                continue
            raise ValueError("cannot remove document root")
        parent = _walk(doc, parts[:-1])
        last = parts[-1]
        if isinstance(parent, list):
            if kind == "add":
                idx = len(parent) if last == "-" else int(last)
                parent.insert(idx, deep_copy(op["value"]))
            elif kind == "replace":
                parent[int(last)] = deep_copy(op["value"])
            elif kind == "remove":
                parent.pop(int(last))
        else:
            if kind in ("add", "replace"):
                if kind == "replace" and last not in parent:
                    raise KeyError(op["path"])
                parent[last] = deep_copy(op["value"])
            elif kind == "remove":
                del parent[last]
    return doc


def apply_patch(live: dict | None, applied: dict) -> dict:
    """Single-manager server-side-apply approximation (see module docstring)."""
    applied = deep_copy(applied)
    if live is None:
        return applied
    out = dict(live)
    for k, v in applied.items():
        if k == "metadata":
            m = dict(live.get("metadata") or {})
            am = v or {}
            for mk in ("labels", "annotations"):
                if mk in am:
                    merged = dict(m.get(mk) or {})
                    merged.update(am[mk] or {})
                    m[mk] = merged
            if "ownerReferences" in am:
                cur = list(m.get("ownerReferences") or [])
                uids = {r.get("uid") for r in cur}
                for r in am["ownerReferences"] or []:
                    if r.get("uid") not in uids:
                        cur.append(r)
                        uids.add(r.get("uid"))
                m["ownerReferences"] = cur
            out["metadata"] = m
        elif k in ("apiVersion", "kind"):
            out[k] = v
        else:
            out[k] = v
    return out
