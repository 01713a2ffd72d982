#!/usr/bin/env python
"""Keep the line references of docs/COMPONENTS.md true to the tree.

A reference is a backticked `path:line` (or `:line`, meaning the last path named before it) followed by a
backticked symbol: `ncc/app.py:671` `main`.  Each must point at the line that defines the symbol (`def`,
`class`, a C++ function/struct/class, or a module-level assignment).  `--fix` rewrites stale line numbers
to the definition nearest the old one; without it, stale or unresolvable references are listed and the
exit status is 1 (tests/test_docs.py runs the check).

    python scripts/doc_refs.py [--fix] [docs/COMPONENTS.md ...]
"""
from __future__ import annotations

import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_TOKEN = re.compile(r"`([\w./-]+\.(?:py|cpp|hpp|yaml))`|"
                    r"`((?:[\w./-]+\.(?:py|cpp|hpp|yaml))?):(\d+)(?:[-–]\d+)?`(?:\s*`([\w.~]+)`)?")


def definitions(path: str, name: str) -> list[int]:
    try:
        with open(os.path.join(ROOT, path)) as f:
            lines = f.read().split("\n")
    except OSError:
        return []
    n = re.escape(name.split(".")[-1])
    pats = [re.compile(rf"^\s*(async\s+)?def {n}\b"), re.compile(rf"^\s*class {n}\b"), re.compile(rf"^{n}\s*[:=]"),
            re.compile(rf"^\s*(struct|class) {n}\b"),
            re.compile(rf"^\s*(static |inline |template <[^>]*> )*[\w:<>,*& ]+[\s*&]{n}\(")]
    return [i + 1 for i, line in enumerate(lines) if any(p.search(line) for p in pats)]


def check(doc_path: str, fix: bool) -> list[str]:
    with open(doc_path) as f:
        doc = f.read()
    problems, edits, cur = [], [], None
    for m in _TOKEN.finditer(doc):
        if m.group(1):  # a bare path: later `:line` references are relative to it
            cur = m.group(1)
            continue
        if m.group(2):
            cur = m.group(2)
        line, name = int(m.group(3)), m.group(4)
        if not name or not cur:
            continue
        hits = definitions(cur, name)
        if not hits:
            problems.append(f"{cur}:{line} `{name}`: no definition found")
        elif line not in hits:
            new = min(hits, key=lambda h: abs(h - line))
            problems.append(f"{cur}:{line} `{name}`: defined at line {new}")
            edits.append((m.start(3), m.end(3), str(new)))
    if fix and edits:
        for start, end, new in sorted(edits, reverse=True):
            doc = doc[:start] + new + doc[end:]
        with open(doc_path, "w") as f:
            f.write(doc)
    return problems


def main(argv=None) -> int:
    args = sys.argv[1:] if argv is None else argv
    fix = "--fix" in args
    docs = [a for a in args if not a.startswith("--")] or [os.path.join(ROOT, "docs", "COMPONENTS.md")]
    bad = []
    for d in docs:
        bad += check(d, fix)
    for p in bad:
        print(p)
    return 0 if fix or not bad else 1


if __name__ == "__main__":
    sys.exit(main())
