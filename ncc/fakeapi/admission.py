"""Server-side mutation of writes: what a real kube-apiserver may store instead of the body it was sent.

A controller that caches its own writes (the native mode's slim caches and echo promotion,
ncc/shards/shard.py `_tracked`, ncc/cache/informer.py `end_write`) must not assume the stored object
equals its request.  Two mechanisms change it on a real cluster, and the fake apiserver can play both:

* CRD structural defaulting and pruning (`prune_defaults`): `default`s of the CRD's schema are filled
  in and unknown fields of non-preserving objects are dropped — e.g. a shard cluster running an older
  or newer NexusAlgorithmTemplate CRD than the controller cluster;
* a mutating admission webhook (`sets`): `{plural: {"dotted.path": value}}` fields written into every
  create/update of that resource (value None deletes the field).

The reference controller compares typed objects with reflect.DeepEqual (controller.go:539,600,725,795):
on such a shard it sees a difference on every pass and issues an update each time (no loop, since an
update that stores the same object is a no-op without a watch event).  Used by
tests/test_server_mutation.py; `python -m ncc.fakeapi --prune-defaults --admission-set ...` and
`POST /_fake/admission` turn it on in a separate fake apiserver process.
"""
from __future__ import annotations

import copy


class Admission:
    def __init__(self):
        self.prune_defaults = False
        self.sets: dict[str, dict[str, object]] = {}
        self.mutated = 0  # writes whose body the webhook changed

    @property
    def active(self) -> bool:
        return self.prune_defaults or bool(self.sets)

    def update(self, d: dict) -> None:
        if "prune_defaults" in d:
            self.prune_defaults = bool(d["prune_defaults"])
        if "sets" in d:
            self.sets = {str(k): dict(v or {}) for k, v in (d["sets"] or {}).items()}

    def as_dict(self) -> dict:
        return {"prune_defaults": self.prune_defaults, "sets": self.sets, "mutated": self.mutated}

    def admit(self, rt, obj: dict, crd: dict | None, subresource: str | None = None) -> None:
        """Mutate a create/update body in place (webhook first, then the schema's defaulting/pruning,
        as the apiserver re-defaults and re-prunes what webhooks return)."""
        fields = self.sets.get(rt.plural) if subresource is None else None
        if fields:
            before = copy.deepcopy(obj)
            for path, value in fields.items():
                _set_path(obj, path.split("."), value)
            if obj != before:
                self.mutated += 1
        if self.prune_defaults and crd is not None:
            from ..api.schema import default_and_prune_object
            default_and_prune_object(crd, obj, rt.version)


def _set_path(obj: dict, path: list, value) -> None:
    cur = obj
    for p in path[:-1]:
        nxt = cur.get(p)
        if not isinstance(nxt, dict):
            if value is None:
                return
            nxt = cur[p] = {}
        cur = nxt
    if value is None:
        cur.pop(path[-1], None)
    else:
        cur[path[-1]] = copy.deepcopy(value)
