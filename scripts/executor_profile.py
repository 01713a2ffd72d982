#!/usr/bin/env python
"""Where the C++ shard executor spends its CPU: symbolizes the executor's own sampling profile.

Run anything that starts executors with `NCC_SAMPLE_PROFILE=<dir>` (optionally `NCC_SAMPLE_US`, default
500 µs of CPU between samples); each executor writes `<dir>/executor-<index>-<pid>.samples` on exit: the
offset, in the executable, of the instruction each SIGPROF interrupted (native/executor/executor.cpp
`start_sampling`).  This maps the offsets to functions with `addr2line -i` and prints these views:

* self — the innermost function at the sample, inlined functions counted as themselves;
* frame — the function whose machine code it is (what an inlined helper was inlined into; coroutine bodies
  show up as their own frames);
* line — the hottest source lines;
* library code by caller — time in libc/libstdc++ leaves (memcpy, system-call wrappers) and library templates by
  the executor's call site: the first of its own functions up the frame-pointer chain (the `profile` build,
  build/profile/ncc-executor), else the return address on top of the stack;
* inclusive (frame-pointer build only) — each of the executor's functions once per sample it is on the stack.

    NCC_SAMPLE_PROFILE=/tmp/prof python bench.py --steps 20 --warmup 5
    python scripts/executor_profile.py /tmp/prof [--binary ncc/bin/ncc-executor] [--top 30]
"""
from __future__ import annotations

import argparse
import collections
import glob
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def local_path(path: str) -> str:
    """`path` itself when it exists here, else the file of this checkout with the longest common tail."""
    if os.path.isfile(path) or not path.startswith("/"):
        return path
    parts = path.strip("/").split("/")
    for i in range(1, len(parts)):
        cand = os.path.join(ROOT, *parts[i:])
        if os.path.isfile(cand):
            return cand
    return path


def load_samples(paths: list[str]) -> collections.Counter:
    """((module, address in the module's file), (module, address) of the top-of-stack word or None when it is not
    code, (call sites up the frame-pointer chain, each (module, return address - 1)...)) -> samples, over every
    process's file.  The chain is empty unless the executor was the frame-pointer build (`build/profile/`)."""
    counts: collections.Counter = collections.Counter()
    for p in paths:
        files = sorted(glob.glob(os.path.join(p, "*.samples"))) if os.path.isdir(p) else [p]
        for f in files:
            maps = []  # (start, end, file offset, path)
            raw: collections.Counter = collections.Counter()
            with open(f) as fh:
                for line in fh:
                    if line.startswith("# map "):
                        parts = line[6:].split()
                        lo, hi = (int(x, 16) for x in parts[0].split("-"))
                        maps.append((lo, hi, int(parts[2], 16), parts[5] if len(parts) > 5 else "[anon]"))
                    elif line.strip():
                        words = [int(w, 16) for w in line.split()]
                        raw[(words[0], words[1] if len(words) > 1 else 0, tuple(words[2:]))] += 1

            def where(addr):
                for lo, hi, off, path in maps:
                    if lo <= addr < hi:
                        return path, addr - lo + off
                return None

            # a profile taken on another machine (the GPU box runs a copy of this tree elsewhere): its files
            # under the repository map to this checkout by their path relative to it
            maps = [(lo, hi, off, local_path(path)) for lo, hi, off, path in maps]

            for (pc, top, chain), n in raw.items():
                sites = tuple(w for w in (where(r - 1) for r in chain) if w is not None)
                counts[(where(pc) or ("[unknown]", pc), where(top), sites)] += n
    return counts


def short(fn: str, width: int = 110) -> str:
    fn = re.sub(r"std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> >", "std::string", fn)
    fn = re.sub(r"std::basic_string_view<char, std::char_traits<char> >", "std::string_view", fn)
    return fn if len(fn) <= width else fn[:width - 3] + "..."


def symbolize(binary: str, addrs: list[int]) -> dict[int, list[tuple[str, str]]]:
    """address -> inline chain [(function, file:line)], innermost first."""
    out: dict[int, list[tuple[str, str]]] = {}
    chunk = 20000
    for lo in range(0, len(addrs), chunk):
        batch = addrs[lo:lo + chunk]
        r = subprocess.run(["addr2line", "-a", "-f", "-C", "-i", "-e", binary], input="\n".join(f"{a:x}" for a in batch),
                           capture_output=True, text=True, check=True)
        cur = None
        lines = r.stdout.splitlines()
        i = 0
        while i < len(lines):
            line = lines[i]
            if line.startswith("0x"):
                cur = int(line, 16)
                out[cur] = []
                i += 1
                continue
            fn = line
            loc = lines[i + 1] if i + 1 < len(lines) else "??:0"
            out[cur].append((fn, os.path.relpath(loc, ROOT) if loc.startswith(ROOT) else loc))
            i += 2
    return out


_IFUNCS = ("memmove", "memcpy", "memset", "memcmp", "bcmp", "memchr", "strlen", "strcmp", "strchr", "rawmemchr")


def exported_spans(lib: str) -> list[tuple[int, int]]:
    """(start, end) of every exported function of a shared library (`nm -D -S`)."""
    try:
        r = subprocess.run(["nm", "-D", "-S", "--defined-only", lib], capture_output=True, text=True, check=True)
    except (OSError, subprocess.CalledProcessError):
        return []
    spans = []
    for line in r.stdout.splitlines():
        w = line.split()
        if len(w) >= 4 and w[2] in ("T", "t", "W", "i"):
            spans.append((int(w[0], 16), int(w[0], 16) + int(w[1], 16)))
    return spans


def ifunc_bodies(lib: str) -> list[tuple[int, str]]:
    """(offset in the library's file, name) of the string/memory routines this machine's dynamic linker picked
    (glibc's IFUNC bodies, e.g. __memmove_avx512_unaligned_erms, are not exported: `nm -D` and addr2line name
    them after the nearest exported symbol, e.g. `__nss_database_lookup`).  Resolved here with dlsym, so the
    report must run on the machine the samples came from (scripts/box/run.sh does)."""
    import ctypes
    try:
        h = ctypes.CDLL(lib)
    except OSError:
        return []
    maps = []
    with open("/proc/self/maps") as f:
        for line in f:
            parts = line.split()
            if len(parts) > 5 and os.path.realpath(parts[5]) == os.path.realpath(lib):
                lo, hi = (int(x, 16) for x in parts[0].split("-"))
                maps.append((lo, hi, int(parts[2], 16)))
    out = []
    for name in _IFUNCS:
        try:
            addr = ctypes.cast(getattr(h, name), ctypes.c_void_p).value
        except AttributeError:
            continue
        for lo, hi, off in maps:
            if lo <= addr < hi:
                out.append((addr - lo + off, name))
    return sorted(set(out))


def relabel_library(path: str, chains: dict) -> None:
    """Names a library sample outside every exported function after the IFUNC body it falls in (the nearest
    picked routine below it, within 8 KiB), else `<lib> internal`."""
    if not os.path.isfile(path):
        return
    spans = exported_spans(path)
    bodies = ifunc_bodies(path) if os.path.basename(path).startswith("libc.") else []
    for (p, a), chain in chains.items():
        if p != path or any(lo <= a < hi for lo, hi in spans):
            continue
        below = [(o, n) for o, n in bodies if o <= a < o + 0x2000]
        if below:
            names = "/".join(n for o, n in bodies if o == max(below)[0])
            chain[:] = [(f"{names} (IFUNC body)", chain[0][1] if chain else "??:0")]
        else:
            chain[:] = [(f"{os.path.basename(path)} internal", chain[0][1] if chain else "??:0")]


_LIB_NAMES = ("std::", "__gnu_cxx::", "void std::", "bool std::", "__gnu_cxx::__enable_if", "operator new",
              "operator delete", "ncc::alloc::")


def _ours(name: str) -> bool:
    """A function of the executor's own code, not a library template instantiated in it."""
    return not name.startswith(_LIB_NAMES)


def report(counts: collections.Counter, binary: str, top: int) -> str:
    total = sum(counts.values())
    if not total:
        return "no samples"
    chains = {}
    modules: collections.Counter = collections.Counter()
    wanted = collections.defaultdict(set)
    rbin = os.path.realpath(binary)
    have_stacks = False
    for (pc, tos, sites), n in counts.items():
        modules[os.path.basename(pc[0])] += n
        wanted[pc[0]].add(pc[1])
        if tos is not None and pc[0] != rbin and tos[0] == rbin:
            wanted[tos[0]].add(tos[1])
        for site in sites:
            have_stacks = True
            if site[0] == rbin:
                wanted[site[0]].add(site[1])
    for path, addrs in wanted.items():
        if os.path.isfile(path):
            for a, chain in symbolize(path, sorted(addrs)).items():
                chains[(path, a)] = chain
            if os.path.realpath(path) != rbin:
                relabel_library(path, chains)
    self_c: collections.Counter = collections.Counter()
    frame_c: collections.Counter = collections.Counter()
    line_c: collections.Counter = collections.Counter()
    lib_c: collections.Counter = collections.Counter()
    incl_c: collections.Counter = collections.Counter()
    for (pc, tos, sites), n in counts.items():
        path = pc[0]
        chain = chains.get(pc) or [("??", "??:0")]
        ours = os.path.realpath(path) == rbin
        tag = "" if ours else f"  [{os.path.basename(path)}]"
        self_c[chain[0][0] + tag] += n
        frame_c[chain[-1][0] + tag] += n
        line_c[f"{chain[0][1].split(' ')[0]}  ({short(chain[0][0], 50)}){tag}"] += n
        # the executor's own call sites up the stack (frame-pointer build), innermost first, inlined callers kept
        up = [c for s in sites for c in (chains.get(s) or [])]
        if not ours or not _ours(chain[-1][0]):  # a leaf in a library or a library template: who called it
            site = next((c for c in up if _ours(c[0])), None)
            if site is not None:
                who = f"{site[1].split(' ')[0]} ({short(site[0], 60)})"
            else:
                caller = chains.get(tos) if tos is not None else None
                who = f"{caller[0][1].split(' ')[0]} ({short(caller[-1][0], 60)})" if caller else "?"
            lib_c[f"{short(chain[0][0], 40)}{tag}  <-  {who}"] += n
        if have_stacks:
            seen = set()
            for fn in [c[0] for c in chain] + [c[0] for c in up]:
                if _ours(fn) and fn not in seen:
                    seen.add(fn)
                    incl_c[fn] += n
    out = [f"{total} samples" + ("" if have_stacks else " (no call stacks: not the frame-pointer build)")]
    out.append("\n== module")
    for name, n in modules.most_common():
        out.append(f"{100.0 * n / total:6.2f}%  {n:7d}  {name}")
    views = [("self (innermost function, inlined code counted as itself)", self_c),
             ("frame (the function whose code ran: inlined helpers folded into their caller)", frame_c),
             ("line", line_c),
             ("library code by caller (the executor's call site that entered it)", lib_c)]
    if have_stacks:
        views.append(("inclusive (the executor's functions on the sampled stack, each once per sample)", incl_c))
    for title, c in views:
        out.append(f"\n== {title}")
        for name, n in c.most_common(top):
            out.append(f"{100.0 * n / total:6.2f}%  {n:7d}  {short(name)}")
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="+", help="NCC_SAMPLE_PROFILE directories or .samples files")
    ap.add_argument("--binary", default=os.path.join(ROOT, "ncc", "bin", "ncc-executor"))
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    text = report(load_samples(a.paths), a.binary, a.top)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
