"""A statistical CPU profiler for the Python processes (coordinator, Python executors), with far less
overhead than cProfile: `NCC_PY_SAMPLE=<path>` arms ITIMER_PROF (every `NCC_PY_SAMPLE_US`, default 1000 µs
of the process's CPU); each SIGPROF records the interrupted Python stack, and at exit the counts go to
`<path>.<role>.<pid>.json`:

    {"samples": n, "self": {"func (file:line)": n}, "inclusive": {"func (file)": n}, "stacks": {"a;b;c": n}}

Python runs signal handlers between bytecodes, so time inside a C call (a native decode, a socket send) is
charged to the Python line that made it — which is where it would be cut anyway.  The C++ executor has
its own sampler (`NCC_SAMPLE_PROFILE`, native/executor/executor.cpp).  With `NCC_NATIVE_SAMPLE=1` too, the
extension records the C++ instruction each tick interrupted (native/ext/sampler.hpp) into
`<path>.<role>.<pid>.native.samples`, which scripts/executor_profile.py symbolizes against the extension
(`--binary ncc/_native*.so`).
"""
from __future__ import annotations

import atexit
import json
import os
import signal
from collections import Counter

_self: Counter = Counter()
_incl: Counter = Counter()
_stacks: Counter = Counter()
_n = [0]


def _where(code, line: int) -> str:
    return f"{code.co_name} ({os.path.basename(code.co_filename)}:{line})"


def _on_prof(signum, frame) -> None:
    if frame is None:
        return
    _n[0] += 1
    _self[_where(frame.f_code, frame.f_lineno)] += 1
    seen = set()
    names = []
    f = frame
    depth = 0
    while f is not None and depth < 40:
        c = f.f_code
        key = f"{c.co_name} ({os.path.basename(c.co_filename)})"
        if key not in seen:
            seen.add(key)
            _incl[key] += 1
        if depth < 8:
            names.append(c.co_name)
        f = f.f_back
        depth += 1
    _stacks[";".join(reversed(names))] += 1


def start(role: str) -> bool:
    path = os.environ.get("NCC_PY_SAMPLE")
    if not path:
        return False
    us = max(100, int(os.environ.get("NCC_PY_SAMPLE_US", "1000")))
    signal.signal(signal.SIGPROF, _on_prof)
    signal.setitimer(signal.ITIMER_PROF, us / 1e6, us / 1e6)

    def dump() -> None:
        signal.setitimer(signal.ITIMER_PROF, 0, 0)
        out = {"samples": _n[0], "interval_us": us,
               "self": dict(_self.most_common(200)), "inclusive": dict(_incl.most_common(200)),
               "stacks": dict(_stacks.most_common(300))}
        try:
            with open(f"{path}.{role}.{os.getpid()}.json", "w") as f:
                json.dump(out, f, indent=0)
        except OSError:
            pass
    atexit.register(dump)
    if os.environ.get("NCC_NATIVE_SAMPLE"):
        # the extension's own time, by C++ function (native/ext/sampler.hpp): what each native line above spends
        from . import native as _native
        mod = _native.load()
        if mod is not None and hasattr(mod, "native_sample_start") and mod.native_sample_start(us):
            nat_path = f"{path}.{role}.{os.getpid()}.native.samples"
            atexit.register(lambda: mod.native_sample_dump(nat_path))
    return True
