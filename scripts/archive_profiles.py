#!/usr/bin/env python
"""Fold old profile directories into one `archive.jsonl` per round, and read them back.

Each round's box runs left hundreds of small files (bench JSON lines, stderr tails, sampling profiles) under
`profiles/rN/<run>/`.  Once a round's numbers are summarised in BENCHMARKS_ARCHIVE.md, its raw files are
packed here — one JSON line per original file, `{"path": "profiles/r2/ab_slim/a_1.json", "json": …}` (or
`"text"` for anything that is not JSON) — so every path the archive cites can still be read, and the tree
keeps a few hundred files instead of 1 300.  Markdown files stay where they are.

    python scripts/archive_profiles.py pack profiles/r2 [--keep r2a,r2b]   # fold everything but --keep
    python scripts/archive_profiles.py show profiles/r2/ab_slim/a_1.json    # print one archived file
    python scripts/archive_profiles.py list profiles/r2 [substring]         # archived paths
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARCHIVE = "archive.jsonl"


def _round_of(path: str) -> str:
    parts = os.path.normpath(path).split(os.sep)
    i = parts.index("profiles")
    return os.path.join(ROOT, *parts[i:i + 2])


def load(round_dir: str) -> dict[str, dict]:
    out = {}
    p = os.path.join(round_dir, ARCHIVE)
    if os.path.exists(p):
        with open(p) as f:
            for line in f:
                if line.strip():
                    rec = json.loads(line)
                    out[rec["path"]] = rec
    return out


def pack(round_dir: str, keep: set[str]) -> tuple[int, int]:
    """Fold every file of `round_dir` (but markdown, the archive itself and the `keep` subdirectories) into
    its archive; returns (files packed, files left)."""
    round_dir = os.path.abspath(round_dir)
    recs = load(round_dir)
    packed, left = [], 0
    for dirpath, dirs, files in os.walk(round_dir):
        rel_dir = os.path.relpath(dirpath, round_dir)
        top = rel_dir.split(os.sep)[0]
        if top in keep:
            left += len(files)
            continue
        for fn in sorted(files):
            full = os.path.join(dirpath, fn)
            if fn == ARCHIVE or fn.endswith(".md"):
                left += 1
                continue
            rel = os.path.relpath(full, ROOT)
            with open(full, "rb") as f:
                raw = f.read()
            text = raw.decode("utf-8", errors="replace")
            try:
                rec = {"path": rel, "json": json.loads(text)}
            except ValueError:
                rec = {"path": rel, "text": text}
            recs[rel] = rec
            packed.append(full)
    with open(os.path.join(round_dir, ARCHIVE + ".tmp"), "w") as f:
        for rel in sorted(recs):
            f.write(json.dumps(recs[rel], separators=(",", ":")) + "\n")
    os.replace(os.path.join(round_dir, ARCHIVE + ".tmp"), os.path.join(round_dir, ARCHIVE))
    for full in packed:
        os.remove(full)
    for dirpath, dirs, files in sorted(os.walk(round_dir), key=lambda t: -len(t[0])):
        if dirpath != round_dir and not os.listdir(dirpath):
            os.rmdir(dirpath)
    return len(packed), left


def show(path: str) -> str:
    rel = os.path.relpath(os.path.abspath(path), ROOT)
    if os.path.exists(os.path.join(ROOT, rel)):
        with open(os.path.join(ROOT, rel)) as f:
            return f.read()
    rec = load(_round_of(os.path.join(ROOT, rel))).get(rel)
    if rec is None:
        raise FileNotFoundError(rel)
    return json.dumps(rec["json"], indent=1) if "json" in rec else rec["text"]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    p = sub.add_parser("pack")
    p.add_argument("round_dir")
    p.add_argument("--keep", default="", help="comma-separated run directories left as they are")
    s = sub.add_parser("show")
    s.add_argument("path")
    ls = sub.add_parser("list")
    ls.add_argument("round_dir")
    ls.add_argument("needle", nargs="?", default="")
    a = ap.parse_args(argv)
    if a.cmd == "pack":
        n, left = pack(a.round_dir, {k for k in a.keep.split(",") if k})
        print(f"packed {n} files into {os.path.join(a.round_dir, ARCHIVE)}; {left} left as files")
    elif a.cmd == "show":
        sys.stdout.write(show(a.path))
    else:
        for rel in load(os.path.abspath(a.round_dir)):
            if a.needle in rel:
                print(rel)
    return 0


if __name__ == "__main__":
    sys.exit(main())
