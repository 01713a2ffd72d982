"""Loader for the in-tree C++ runtime extension `ncc._native`.

The extension (sources in `native/`, built in-tree by `python native/build.py` or
`__graft_entry__.build()`) provides the hot runtime primitives the reference gets from
compiled client-go — the rate-limited exclusive-key work queue and structural fingerprints
used for O(1) drift detection — plus the per-object hot spots of
this runtime: watch-line/response scanners with crc32 key partitions, a compact JSON encoder
and HTTP/1.1 head parsers (see the header of native/ncc_native.cpp).

`load(required=False)` returns the module or None.  Set `NCC_REQUIRE_NATIVE=1` (the GPU-box
test tier does) to turn a missing or stale build into a hard ImportError instead of a silent
Python fallback.
"""
from __future__ import annotations

import os

_mod = None
_err: BaseException | None = None
ABI_VERSION = 33  # bump together with NCC_NATIVE_ABI in native/ncc_native.cpp


def load(required: bool = False):
    global _mod, _err
    if _mod is None and _err is None:
        try:
            from .. import _native as m  # type: ignore[attr-defined]
            if getattr(m, "ABI_VERSION", None) != ABI_VERSION:
                raise ImportError(f"ncc._native ABI {getattr(m, 'ABI_VERSION', None)} != expected {ABI_VERSION}; "
                                  f"rebuild with `python native/build.py`")
            _mod = m
        except ImportError as e:
            _err = e
    if _mod is None and (required or os.environ.get("NCC_REQUIRE_NATIVE") == "1"):
        raise ImportError(f"ncc._native extension is required but unavailable: {_err}")
    return _mod


def available() -> bool:
    return load() is not None
