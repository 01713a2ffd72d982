"""Compact JSON encoding (and UTF-8 decoding) for request bodies, responses and watch lines.

Uses the native encoder (`ncc._native.dumps`, ~4x faster than `json.dumps` on Kubernetes objects)
when the extension is built, else the standard library.  Output is compact (`,`/`:` separators) with
key order preserved; the native path writes non-ASCII text as UTF-8 instead of `\\u` escapes — both
are valid JSON and decode identically.
"""
from __future__ import annotations

import json

from .. import native as _native

_mod = _native.load()
_native_dumps = getattr(_mod, "dumps", None) if _mod is not None else None


_decode = json.JSONDecoder().decode


def loads_bytes(b):
    """json.loads for UTF-8 wire bytes (Kubernetes JSON is always UTF-8) without the stdlib's per-call
    encoding detection."""
    return _decode(b.decode("utf-8", "surrogatepass") if isinstance(b, (bytes, bytearray, memoryview)) else b)


_native_loads = getattr(_mod, "loads", None) if _mod is not None else None


def loads_fast(b):
    """`loads_bytes` through the native decoder (`ncc._native.loads`, ~2x the stdlib on Kubernetes objects)
    when it is built; anything it does not accept (malformed input, NaN/Infinity literals) is left to the
    stdlib, which also raises the proper error.  The controller's hot decode path; the fake apiservers (the
    test substrate) keep the stdlib decoder."""
    if _native_loads is not None and isinstance(b, bytes):
        v = _native_loads(b)
        if v is not None:
            return v
    return loads_bytes(b)


def dumps_bytes(obj) -> bytes:
    if _native_dumps is not None:
        try:
            return _native_dumps(obj)
        except (TypeError, ValueError):
            pass  # non-JSON-shaped input (e.g. non-string keys): the stdlib decides
    return json.dumps(obj, separators=(",", ":")).encode()
