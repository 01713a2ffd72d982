#!/usr/bin/env python
"""Line-coverage gate for the `ncc` package, stdlib only (no coverage.py in this image).

Mirrors the reference CI's coverage gate (.testcoverage.yml:5-8: 70 % per file, 70 % per package,
75 % total) for this codebase: runs the CPU test tier in-process under a `sys.settrace` line
collector restricted to `ncc/`, then compares executed lines against every line that carries
bytecode (from the compiled code objects).  Subprocesses (executors, fake apiservers spawned by
tests) are not traced, so files only exercised there are listed but exempt via --exempt.

    python scripts/coverage_gate.py                 # report + gate (exit 1 below thresholds)
    python scripts/coverage_gate.py --report-only   # just the table
"""
from __future__ import annotations

import argparse
import os
import sys
import threading
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ncc") + os.sep

# Run only by child processes (executor/fakeapi entry points) or pure CLI glue.
DEFAULT_EXEMPT = ("ncc/__main__.py", "ncc/executor.py", "ncc/fakeapi/__main__.py")


def executable_lines(path: str) -> set[int]:
    with open(path, "rb") as f:
        src = f.read()
    try:
        code = compile(src, path, "exec")
    except SyntaxError:
        return set()
    lines: set[int] = set()
    stack = [code]
    while stack:
        co = stack.pop()
        for _, _, ln in co.co_lines():
            if ln is not None:
                lines.add(ln)
        stack.extend(c for c in co.co_consts if hasattr(c, "co_lines"))
    # docstring-only / def lines of the module body count once they import; keep everything else
    return lines


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--file", type=float, default=70.0)
    ap.add_argument("--package", type=float, default=70.0)
    ap.add_argument("--total", type=float, default=75.0)
    ap.add_argument("--exempt", action="append", default=list(DEFAULT_EXEMPT))
    ap.add_argument("--report-only", action="store_true")
    ap.add_argument("--show-missing", action="append", default=[], metavar="FILE",
                    help="print the unexecuted line ranges of FILE (repo-relative, e.g. ncc/fakeapi/server.py)")
    ap.add_argument("pytest_args", nargs="*", default=["tests", "-q", "-x", "-m", "not gpu", "-p", "no:cacheprovider"])
    a = ap.parse_args(argv)

    hits: dict[str, set[int]] = defaultdict(set)

    def local(frame, event, arg):
        if event == "line":
            hits[frame.f_code.co_filename].add(frame.f_lineno)
        return local

    def glob(frame, event, arg):
        fn = frame.f_code.co_filename
        if fn.startswith(PKG):
            hits[fn].add(frame.f_lineno)
            return local
        return None

    sys.path.insert(0, ROOT)
    import pytest
    threading.settrace(glob)
    sys.settrace(glob)
    try:
        rc = pytest.main(a.pytest_args)
    finally:
        sys.settrace(None)
        threading.settrace(None)
    if rc != 0:
        print(f"tests failed (pytest exit {rc}); coverage not evaluated", file=sys.stderr)
        return int(rc)

    rows = []
    missing: dict[str, list[int]] = {}
    pkg_tot: dict[str, list[int]] = defaultdict(lambda: [0, 0])
    tot = [0, 0]
    for dirpath, _, files in os.walk(PKG):
        for f in sorted(files):
            if not f.endswith(".py"):
                continue
            path = os.path.join(dirpath, f)
            rel = os.path.relpath(path, ROOT)
            exe = executable_lines(path)
            if not exe:
                continue
            got = len(exe & hits.get(path, set()))
            pkg = os.path.dirname(rel)
            exempt = rel in a.exempt
            rows.append((rel, got, len(exe), exempt))
            if rel in a.show_missing:
                missing[rel] = sorted(exe - hits.get(path, set()))
            if not exempt:
                pkg_tot[pkg][0] += got
                pkg_tot[pkg][1] += len(exe)
                tot[0] += got
                tot[1] += len(exe)
    bad = []
    print(f"\n{'file':52s} {'cov':>7s}  lines")
    for rel, got, n, exempt in sorted(rows):
        pct = 100.0 * got / n
        flag = " (exempt)" if exempt else ("  < gate" if pct < a.file else "")
        if not exempt and pct < a.file:
            bad.append(f"file {rel} {pct:.1f}%")
        print(f"{rel:52s} {pct:6.1f}%  {got}/{n}{flag}")
    print()
    for pkg, (got, n) in sorted(pkg_tot.items()):
        pct = 100.0 * got / n
        if pct < a.package:
            bad.append(f"package {pkg} {pct:.1f}%")
        print(f"package {pkg:44s} {pct:6.1f}%")
    total = 100.0 * tot[0] / max(tot[1], 1)
    print(f"\nTOTAL {total:.1f}%  ({tot[0]}/{tot[1]} lines)")
    for rel, ls in missing.items():
        spans, start = [], None
        for i, ln in enumerate(ls):
            if start is None:
                start = ln
            if i + 1 == len(ls) or ls[i + 1] != ln + 1:
                spans.append(f"{start}" if start == ln else f"{start}-{ln}")
                start = None
        print(f"missing {rel}: {', '.join(spans)}")
    if total < a.total:
        bad.append(f"total {total:.1f}%")
    if bad and not a.report_only:
        print("coverage gate FAILED: " + "; ".join(bad), file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
