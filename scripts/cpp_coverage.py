#!/usr/bin/env python
"""Line-coverage gate for the C++ shard executor (native/executor/), with gcov.

The Python gate (scripts/coverage_gate.py) cannot see the C++ data plane that native mode runs by default.
This builds `ncc/bin/ncc-executor` with gcov instrumentation (`native/build.py --executor-coverage`: -O0
--coverage; the executor flushes its counters on exit), runs the CPU test tier — every test that starts
the controller in native mode spawns the C++ executor (tests/test_conformance.py runs each scenario against
it; tests/test_native_executor_direct.py drives it over its socketpair protocol) — and reports executed /
executable lines per source file.  It gates `executor.cpp` (default 70 %, the reference CI's per-file bar,
.testcoverage.yml:5-8) and restores the release build afterwards.

    python scripts/cpp_coverage.py                      # build, test, report, gate
    python scripts/cpp_coverage.py --out profiles/r3/executor_gcov.txt
    python scripts/cpp_coverage.py -- tests/test_conformance.py -k native   # a subset
"""
from __future__ import annotations

import argparse
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "ncc", "bin")
SRC = os.path.join(ROOT, "native", "executor")
_LINE = re.compile(r"^\s*([^:]+):\s*(\d+):(.*)$")


def line_sets(path: str) -> tuple[str, set, set]:
    """(source, executable line numbers, executed line numbers) of one .gcov file; a line of a template counts as
    executed when any of its instantiations ran."""
    source, exe, hit = "", set(), set()
    with open(path, errors="replace") as f:
        for raw in f:
            m = _LINE.match(raw)
            if not m:
                continue
            count, lineno = m.group(1).strip(), int(m.group(2))
            if lineno == 0:
                if m.group(3).startswith("Source:"):
                    source = m.group(3)[len("Source:"):]
                continue
            if count == "-":
                continue
            exe.add(lineno)
            if not (count.startswith("#####") or count.startswith("=====")):
                hit.add(lineno)
    return source, exe, hit


def ranges(nums: list[int]) -> str:
    out, start, prev = [], None, None
    for n in nums:
        if start is None:
            start = prev = n
        elif n == prev + 1:
            prev = n
        else:
            out.append(f"{start}-{prev}" if prev != start else str(start))
            start = prev = n
    if start is not None:
        out.append(f"{start}-{prev}" if prev != start else str(start))
    return ",".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--min", type=float, default=70.0, help="line coverage gate for executor.cpp (percent)")
    ap.add_argument("--out", default=None, help="write the report here too")
    ap.add_argument("--keep-build", action="store_true", help="leave the instrumented executor in place")
    ap.add_argument("pytest_args", nargs="*",
                    default=["tests", "-q", "-m", "not gpu", "-n", "8", "-p", "no:cacheprovider"])
    a = ap.parse_args(argv)

    sys.path.insert(0, os.path.join(ROOT, "native"))
    import build as native_build  # native/build.py

    tools = os.path.dirname(native_build.tool_path())
    for f in glob.glob(os.path.join(BIN, "*.gcda")) + glob.glob(os.path.join(BIN, "*.gcno")) + \
            glob.glob(os.path.join(tools, "*.gcda")) + glob.glob(os.path.join(tools, "*.gcno")):
        os.remove(f)
    native_build.build_executor(coverage=True, verbose=True)
    # the executor's HTTP/2 client also runs inside the test tool ncc-h2probe (the RFC 9113 error-code and
    # interop tests drive it): instrumented too, and its counts merged per source line
    native_build.build_tool("ncc-h2probe", verbose=True, coverage=True)
    env = dict(os.environ, NCC_SKIP_NATIVE_BUILD="1")
    env.pop("NCC_EXECUTOR_IMPL", None)
    rc = subprocess.call([sys.executable, "-m", "pytest", *a.pytest_args], cwd=ROOT, env=env)
    gcda = glob.glob(os.path.join(BIN, "*.gcda"))
    report = []
    ok = True
    try:
        if rc != 0:
            report.append(f"pytest failed (exit {rc}); coverage below is of a partial run")
            ok = False
        if not gcda:
            print("no .gcda counters were written: did any test run the C++ executor?", file=sys.stderr)
            return 1
        merged: dict = {}  # source -> (executable lines, executed lines), over the executor and the tool
        for obj_dir, counters in ((BIN, gcda), (tools, glob.glob(os.path.join(tools, "*.gcda")))):
            if not counters:
                continue
            work = os.path.join(obj_dir, "gcov")
            os.makedirs(work, exist_ok=True)
            subprocess.run(["gcov", "-p", "-o", obj_dir, *counters], cwd=work, check=True, stdout=subprocess.DEVNULL)
            for g in sorted(glob.glob(os.path.join(work, "*.gcov"))):
                source, exe, hit = line_sets(g)
                full = os.path.normpath(source if os.path.isabs(source) else os.path.join(ROOT, source))
                if not full.startswith(SRC):
                    continue
                e0, h0 = merged.setdefault(os.path.relpath(full, ROOT), (set(), set()))
                e0 |= exe
                h0 |= hit
        rows = []
        for name in sorted(merged):
            exe, hit = merged[name]
            rows.append((name, len(exe), len(exe & hit), sorted(exe - hit)))
        report.append(f"{'file':<36} {'lines':>7} {'hit':>7} {'cover':>7}")
        gate = None
        for name, total, hit, missing in rows:
            pct = 100.0 * hit / total if total else 100.0
            report.append(f"{name:<36} {total:>7} {hit:>7} {pct:>6.1f}%")
            if name.endswith("executor.cpp"):
                gate = (pct, missing)
        tot = sum(r[1] for r in rows)
        hits = sum(r[2] for r in rows)
        report.append(f"{'total':<36} {tot:>7} {hits:>7} {100.0 * hits / max(tot, 1):>6.1f}%")
        for name, total, hit, missing in rows:
            if missing and not name.endswith("executor.cpp"):
                report.append(f"{os.path.basename(name)} unexecuted lines: {ranges(missing)}")
        if gate is None:
            report.append("executor.cpp: no coverage data")
            ok = False
        else:
            report.append(f"executor.cpp unexecuted lines: {ranges(gate[1])}")
            if gate[0] < a.min:
                report.append(f"FAIL: executor.cpp line coverage {gate[0]:.1f}% < {a.min:.0f}%")
                ok = False
            else:
                report.append(f"OK: executor.cpp line coverage {gate[0]:.1f}% >= {a.min:.0f}%")
        text = "\n".join(report)
        print(text)
        if a.out:
            os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
            with open(a.out, "w") as f:
                f.write(text + "\n")
    finally:
        if not a.keep_build:
            import shutil
            for f in glob.glob(os.path.join(BIN, "*.gcda")) + glob.glob(os.path.join(BIN, "*.gcno")) + \
                    glob.glob(os.path.join(tools, "*.gcda")) + glob.glob(os.path.join(tools, "*.gcno")):
                os.remove(f)
            shutil.rmtree(os.path.join(BIN, "gcov"), ignore_errors=True)
            shutil.rmtree(os.path.join(tools, "gcov"), ignore_errors=True)
            native_build.build_executor()  # the release build back in place
            native_build.build_tool("ncc-h2probe", force=True)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
