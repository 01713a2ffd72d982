"""Loader for the fake apiserver's extension `ncc.fakeapi._native` (sources in native/fakeapi/, built in-tree by
`python native/build.py`): its HTTP/1.1 request-head parser and HTTP/2 server framing.  Test and benchmark
substrate — kept out of the controller's own extension `ncc._native`."""
from __future__ import annotations

_mod = None
_err: BaseException | None = None
ABI_VERSION = 1  # bump together with NCC_FAKEAPI_NATIVE_ABI in native/fakeapi/fakeapi_native.cpp


def load(required: bool = False):
    global _mod, _err
    if _mod is None and _err is None:
        try:
            from . import _native as m  # type: ignore[attr-defined]
            if getattr(m, "ABI_VERSION", None) != ABI_VERSION:
                raise ImportError(f"ncc.fakeapi._native ABI {getattr(m, 'ABI_VERSION', None)} != expected "
                                  f"{ABI_VERSION}; rebuild with `python native/build.py`")
            _mod = m
        except ImportError as e:
            _err = e
    if _mod is None and required:
        raise ImportError(f"ncc.fakeapi._native is required but unavailable: {_err}")
    return _mod


def __getattr__(name: str):
    """`native.H2ServerParser` etc.: the extension's attributes (tests use them directly)."""
    return getattr(load(required=True), name)
