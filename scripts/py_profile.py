"""Report of the Python processes' sampling profiles (`NCC_PY_SAMPLE`, ncc/sampler.py): for each
`<path>.<role>.<pid>.json`, the sample count and the top self lines, then the top inclusive functions over every
file of the same role.  Time inside a native call is charged to the Python line that made it (ncc/sampler.py).

    python scripts/py_profile.py gpurun_out/r6e/py.*.json [--top 20]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys


def load(paths: list[str]) -> list[tuple[str, dict]]:
    out = []
    for p in sorted(paths):
        try:
            with open(p) as f:
                out.append((p, json.load(f)))
        except (OSError, ValueError) as e:
            print(f"skipped {p}: {e}", file=sys.stderr)
    return out


def role_of(path: str) -> str:
    parts = os.path.basename(path).split(".")
    return parts[1] if len(parts) >= 4 else "?"


def report(files: list[tuple[str, dict]], top: int) -> str:
    lines = []
    by_role: dict[str, collections.Counter] = collections.defaultdict(collections.Counter)
    n_role: collections.Counter = collections.Counter()
    for p, d in files:
        n = d.get("samples", 0)
        lines.append(f"## {os.path.basename(p)} — {n} samples (SIGPROF, interval {d.get('interval_us')} µs requested)")
        lines.append("")
        lines.append("self %  | where")
        for where, c in sorted(d.get("self", {}).items(), key=lambda kv: -kv[1])[:top]:
            lines.append(f"{100.0 * c / max(n, 1):6.1f} | {where}")
        lines.append("")
        by_role[role_of(p)].update(d.get("inclusive", {}))
        n_role[role_of(p)] += n
    for role, cnt in by_role.items():
        n = n_role[role]
        lines.append(f"## inclusive, every {role} process — {n} samples")
        lines.append("")
        lines.append("incl % | function")
        for where, c in cnt.most_common(top):
            lines.append(f"{100.0 * c / max(n, 1):6.1f} | {where}")
        lines.append("")
    return "\n".join(lines)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("paths", nargs="+")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args(argv)
    files = load(a.paths)
    if not files:
        print("no profiles")
        return 1
    print(report(files, a.top))
    return 0


if __name__ == "__main__":
    sys.exit(main())
