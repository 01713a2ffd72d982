"""Label-selector parsing and matching (k8s.io/apimachinery/pkg/labels subset).

Supports equality-based (`a=b`, `a==b`, `a!=b`) and set-based (`a in (x,y)`, `a notin (x)`,
`a`, `!a`) requirements joined by commas.  Used by the fake apiserver's list/watch and by
the orphan sweep, which selects shard objects by the `configuration-owner` label.
"""
from __future__ import annotations

import re
from typing import Callable

_SET_RE = re.compile(r"^\s*([A-Za-z0-9_./-]+)\s+(in|notin)\s+\(([^)]*)\)\s*$")


def _split_top(sel: str) -> list[str]:
    parts, depth, cur = [], 0, []
    for ch in sel:
        if ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "," and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(ch)
    if cur:
        parts.append("".join(cur))
    return [p.strip() for p in parts if p.strip()]


def parse(selector: str | None) -> Callable[[dict], bool]:
    """Compile a selector string into a predicate over a label dict."""
    if not selector:
        return lambda _labels: True
    reqs: list[Callable[[dict], bool]] = []
    for part in _split_top(selector):
        m = _SET_RE.match(part)
        if m:
            key, op, vals = m.group(1), m.group(2), {v.strip() for v in m.group(3).split(",") if v.strip()}
            if op == "in":
                reqs.append(lambda l, k=key, vs=vals: l.get(k) in vs)
            else:
                reqs.append(lambda l, k=key, vs=vals: l.get(k) not in vs)
        elif "!=" in part:
            k, v = (s.strip() for s in part.split("!=", 1))
            reqs.append(lambda l, k=k, v=v: l.get(k) != v)
        elif "==" in part:
            k, v = (s.strip() for s in part.split("==", 1))
            reqs.append(lambda l, k=k, v=v: l.get(k) == v)
        elif "=" in part:
            k, v = (s.strip() for s in part.split("=", 1))
            reqs.append(lambda l, k=k, v=v: l.get(k) == v)
        elif part.startswith("!"):
            k = part[1:].strip()
            reqs.append(lambda l, k=k: k not in l)
        else:
            reqs.append(lambda l, k=part: k in l)
    return lambda labels: all(r(labels or {}) for r in reqs)


def from_dict(labels: dict) -> str:
    return ",".join(f"{k}={v}" for k, v in sorted(labels.items()))
