#!/usr/bin/env python
"""Host-side profile of one bench run: cProfile every process (coordinator, executors, fake apiservers)
and write a Markdown summary (top functions by self time, per-module shares).

    python scripts/host_profile.py --out profiles/r1/host_profiles.md [--steps 6] [--executors-per-shard 1]
"""
from __future__ import annotations

import argparse
import collections
import glob
import io
import os
import pstats
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def summarise(path: str, top: int) -> str:
    st = pstats.Stats(path)
    total = sum(v[2] for v in st.stats.values())
    idle = sum(v[2] for k, v in st.stats.items() if k[2] == "<method 'poll' of 'select.epoll' objects>")
    by_mod = collections.Counter()
    for (fn, _ln, _name), (_cc, _nc, tt, _ct, _callers) in st.stats.items():
        if "/repo/" in fn:
            key = fn.split("/repo/")[-1]
        elif "python3" in fn:
            key = "stdlib:" + fn.split("/")[-1]
        else:
            key = fn
        by_mod[key] += tt
    by_mod["~"] -= idle
    by_mod["builtins/C (json, dict, socket, native ext; excl. epoll idle)"] = by_mod.pop("~", 0.0)
    out = io.StringIO()
    busy = max(total - idle, 1e-9)
    out.write(f"total {total:.2f} s, event-loop idle {idle:.2f} s, busy {busy:.2f} s\n\n")
    out.write("| module | self s | % of busy |\n|---|---|---|\n")
    for k, v in by_mod.most_common(12):
        out.write(f"| `{k}` | {v:.3f} | {100 * v / busy:.1f} |\n")
    s = io.StringIO()
    st.stream = s
    st.sort_stats("tottime").print_stats(top)
    lines = [ln for ln in s.getvalue().splitlines() if ln.strip()]
    start = next((i for i, ln in enumerate(lines) if ln.strip().startswith("ncalls")), 0)
    out.write("\n```\n" + "\n".join(lines[start:]) + "\n```\n")
    return out.getvalue()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--templates", type=int, default=1000)
    ap.add_argument("--executors-per-shard", type=int, default=0)
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args(argv)
    d = tempfile.mkdtemp(prefix="ncc-hostprof-")
    env = dict(os.environ, NCC_FAKEAPI_PROFILE=os.path.join(d, "fakeapi"))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup", "1",
           "--templates", str(a.templates), "--extra-env", f"NCC_PROFILE={os.path.join(d, 'ncc')}"]
    if a.executors_per_shard:
        cmd += ["--extra-env", f"NEXUS__EXECUTORS_PER_SHARD={a.executors_per_shard}"]
    res = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    line = (res.stdout.strip().splitlines() or [""])[-1]
    parts = [f"# Host profiles (cProfile) of one `bench.py` run\n\nCommand: `{' '.join(cmd[1:])}` "
             f"(profiling roughly doubles per-call cost; use shares, not absolute times).\n\nBench line: "
             f"`{line[:400]}`\n"]
    names = [("coordinator (python -m ncc)", os.path.join(d, "ncc"))]
    names += [(f"executor {os.path.basename(p).split('executor')[-1]}", p)
              for p in sorted(glob.glob(os.path.join(d, "ncc.executor*")))]
    names += [(f"fake apiserver `{os.path.basename(p).split('.', 1)[1]}`", p)
              for p in sorted(glob.glob(os.path.join(d, "fakeapi.*")))]
    for title, p in names:
        if os.path.exists(p):
            parts.append(f"\n## {title}\n\n" + summarise(p, a.top))
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        f.write("\n".join(parts))
    print(f"wrote {a.out}")
    return 0 if res.returncode == 0 else res.returncode


if __name__ == "__main__":
    sys.exit(main())
