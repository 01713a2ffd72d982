"""Structural fingerprints of JSON-shaped values for O(1) drift detection.

`fingerprint(v)` is a 64-bit digest of the canonical form of `v` (dict keys sorted, type-tagged
scalars), so two values are equal as JSON iff (modulo 2^-64 collisions) their fingerprints are
equal.  It replaces the reference's per-comparison `reflect.DeepEqual` (controller.go:539,600,
725,795) on the slim shard caches, where only the digest of a shard object's `spec`/`data` is
kept instead of the body.

The C++ implementation (`ncc._native.fingerprint`) walks the Python objects directly; the
Python fallback hashes canonical JSON with blake2b and yields *different* digests, so a
process must use one implementation consistently (`IMPL` tells which).
"""
from __future__ import annotations

import hashlib
import json

from .. import native as _native

SLIM_FP = "__ncc_fp__"  # key under which slim-cache transforms store content digests
SLIM_STATUS_FP = "__ncc_sfp__"  # a slim template's digest of its status text (_native.template_event_slim)
# On a slim object published from our own write whose stored payload differs from what we sent (the
# server defaulted, pruned or a webhook mutated it): the digests of what we sent.  That version counts as
# in sync for exactly that intent; any later version (a new watch event, a relist) replaces the object
# and the mark with it, so drift made by others is still seen.
SLIM_WROTE = "__ncc_wrote__"


def _py_fingerprint(v) -> int:
    b = json.dumps(v, sort_keys=True, separators=(",", ":"), ensure_ascii=False).encode()
    return int.from_bytes(hashlib.blake2b(b, digest_size=8).digest(), "little")


_mod = _native.load()
if _mod is not None:
    fingerprint = _mod.fingerprint
    IMPL = "native"
else:  # pragma: no cover - exercised when the extension is not built
    fingerprint = _py_fingerprint
    IMPL = "python"


def content_fingerprint(obj: dict, fields: tuple) -> int:
    """Digest of the given top-level fields of `obj` (missing/empty fields count as empty)."""
    return fingerprint([obj.get(f) or None for f in fields])
