#!/usr/bin/env python
"""Build the in-tree native code: the extension `ncc/_native*.so` (C++17 + pybind11) and the native
shard executor `ncc/bin/ncc-executor` (C++20 coroutines + epoll + OpenSSL, sources in native/executor/) — the
product — and, for tests and benchmarks, the fake apiserver's extension `ncc/fakeapi/_native*.so`
(native/fakeapi/) and the test tool `build/tools/ncc-h2probe` (native/tools/).

Usage: python native/build.py [--debug] [--sanitize] [--product-only]
`--sanitize` builds with AddressSanitizer/UBSan for host-side testing; run the tests with
  NCC_SKIP_NATIVE_BUILD=1 ASAN_OPTIONS=detect_leaks=0 \
  LD_PRELOAD="$(g++ -print-file-name=libasan.so) $(g++ -print-file-name=libstdc++.so)" python -m pytest ...
(libstdc++ must be preloaded too, or ASan's __cxa_throw interceptor cannot resolve the real symbol).
"""
from __future__ import annotations

import argparse
import os
import platform
import shlex
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SOURCES = [os.path.join(HERE, "ncc_native.cpp")]
COMMON_HEADERS = [os.path.join(HERE, "common", f) for f in ("byte_scan.hpp", "hpack.hpp")]  # shared with the executor
# the extension's parts by concern (ncc_native.cpp includes them in order)
EXT_HEADERS = sorted(os.path.join(HERE, "ext", f) for f in os.listdir(os.path.join(HERE, "ext")) if f.endswith(".hpp"))


def _werror() -> list:
    """NCC_WERROR=1 (the CI lint job): warnings fail the build."""
    return ["-Werror"] if os.environ.get("NCC_WERROR") == "1" else []


def arch_flags(machine: str | None = None) -> list:
    """-mpopcnt on x86-64 only: the JSON block scanner counts bracket bits (native/common/byte_scan.hpp) and
    every x86-64 CPU since 2008 has the instruction; other targets (aarch64: the arm64 image) lower
    `__builtin_popcountll` natively and reject the option."""
    m = (machine or os.environ.get("NCC_TARGET_MACHINE") or platform.machine()).lower()
    return ["-mpopcnt"] if m in ("x86_64", "amd64", "x64") else []


def target_path() -> str:
    return os.path.join(ROOT, "ncc", "_native" + sysconfig.get_config_var("EXT_SUFFIX"))


EXECUTOR_DIR = os.path.join(HERE, "executor")
EXECUTOR_MAIN = os.path.join(EXECUTOR_DIR, "executor.cpp")


def executor_path() -> str:
    return os.path.join(ROOT, "ncc", "bin", "ncc-executor")


def build_executor(debug: bool = False, sanitize: bool = False, verbose: bool = False, out: str | None = None,
                   coverage: bool = False, profile: bool = False) -> str:
    """The native shard executor (one translation unit; headers alongside); `out` overrides the in-tree
    path (setup.py builds it into the wheel's ncc/bin/).  `coverage`: gcov instrumentation (the executor
    flushes its counters on exit; scripts/cpp_coverage.py gates the line coverage).  `profile`: the release
    build with frame pointers, so the sampling profiler (NCC_SAMPLE_PROFILE) records call stacks
    (profile_executor_path(); scripts/box/run.sh `sample` runs it)."""
    out = out or (profile_executor_path() if profile else executor_path())
    flavor = "coverage" if coverage else ("sanitize" if sanitize else ("debug" if debug else
                                                                      ("profile" if profile else "release")))
    stamp = out + ".flavor"
    sources = [os.path.join(EXECUTOR_DIR, f) for f in sorted(os.listdir(EXECUTOR_DIR))
               if f.endswith((".cpp", ".hpp"))]
    if os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            same = f.read().strip() == flavor
        if same and all(os.path.getmtime(s) <= os.path.getmtime(out) for s in sources + COMMON_HEADERS + [__file__]):
            return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    flags = ["-std=c++20", "-fcoroutines", *arch_flags(), "-Wall", "-Wextra", "-Wno-unused-parameter", "-g"] + _werror()
    if coverage:
        flags += ["-O0", "--coverage", "-DNCC_COVERAGE", "-DNCC_SYSTEM_MALLOC"]
    elif debug or sanitize:
        flags += ["-O1", "-fno-omit-frame-pointer"]
    else:
        flags += ["-O2", "-DNDEBUG"]
    if profile:
        flags += ["-fno-omit-frame-pointer", "-mno-omit-leaf-frame-pointer", "-DNCC_FRAME_POINTERS"]
    if sanitize:
        # ASan must see every heap allocation: keep malloc instead of the executor's pool allocator
        flags += ["-fsanitize=address,undefined", "-DNCC_SYSTEM_MALLOC"]
    tmp = out + ".tmp"
    cmd = [cxx, *flags, EXECUTOR_MAIN, "-o", tmp, "-lssl", "-lcrypto"]
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(flavor)
    return out


TOOLS_DIR = os.path.join(HERE, "tools")


def profile_executor_path() -> str:
    """The frame-pointer build of the executor for sampling profiles (build/, git-ignored; never shipped)."""
    return os.path.join(ROOT, "build", "profile", "ncc-executor")


def tool_path(name: str = "ncc-h2probe") -> str:
    """Test tools live outside the package (build/tools/, git-ignored): nothing under ncc/ ships them."""
    return os.path.join(ROOT, "build", "tools", name)


TOOLS = {  # test-only programs (build/tools/): name -> (source, extra flags, libraries)
    "ncc-h2probe": ("h2probe.cpp", ["-fcoroutines", "-DNCC_SYSTEM_MALLOC"], ["-lssl", "-lcrypto"]),
    "ncc-strmap-check": ("strmap_check.cpp", [], []),
}


def build_tool(name: str, verbose: bool = False, coverage: bool = False, force: bool = False) -> str:
    """One test tool of TOOLS, rebuilt when it or an executor header changed (`coverage`: gcov-instrumented,
    for scripts/cpp_coverage.py; `force`: rebuilt regardless, e.g. to put the plain build back)."""
    source, flags, libs = TOOLS[name]
    out = tool_path(name)
    src = os.path.join(TOOLS_DIR, source)
    deps = [src] + [os.path.join(EXECUTOR_DIR, f) for f in os.listdir(EXECUTOR_DIR) if f.endswith(".hpp")]
    if not (coverage or force) and os.path.exists(out) and \
            all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps + COMMON_HEADERS):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cxx = os.environ.get("CXX", "g++")
    tmp = out + ".tmp"
    opt = ["-g", "-O0", "--coverage", "-DNCC_COVERAGE"] if coverage else ["-O1"]
    cmd = [cxx, "-std=c++20", *flags, *arch_flags(), "-Wall", "-Wextra", "-Wno-unused-parameter", *opt,
           *_werror(), src, "-o", tmp, *libs]
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


def build_tools(verbose: bool = False) -> str:
    """The test tools: ncc-h2probe (native/tools/h2probe.cpp: the executor's HTTP client, native/executor/http.hpp,
    driven from stdin, for tests against scripted and independent HTTP/2 servers) and ncc-strmap-check (the
    executor's open-addressing map against std::unordered_map).  Test-only; not part of the product.  Returns
    ncc-h2probe's path."""
    for name in TOOLS:
        if name != "ncc-h2probe":
            build_tool(name, verbose)
    return build_tool("ncc-h2probe", verbose)


def build(debug: bool = False, sanitize: bool = False, verbose: bool = False, substrate: bool = True) -> str:
    """The extension first (the relay and the report table need it), then the C++ executor.  A host that
    cannot build the executor (no libssl-dev, no C++20 coroutines) still gets a working package: native mode
    falls back to the Python executor, with a warning here.  NCC_WERROR=1 or NCC_REQUIRE_EXECUTOR=1 (CI, the
    container image) make that failure fatal.  `substrate`: also the fake apiserver's extension (tests,
    benchmarks; the container image builds without it)."""
    out = build_extension(debug, sanitize, verbose)
    if substrate:
        build_extension(debug, sanitize, verbose, sources=FAKEAPI_SOURCES, out=fakeapi_path())
    try:
        build_executor(debug, sanitize, verbose)
    except (subprocess.CalledProcessError, OSError) as e:
        if os.environ.get("NCC_WERROR") == "1" or os.environ.get("NCC_REQUIRE_EXECUTOR") == "1":
            raise
        print(f"warning: the native shard executor was not built ({e}); native mode will use the Python "
              f"executor", file=sys.stderr)
    return out


FAKEAPI_SOURCES = [os.path.join(HERE, "fakeapi", "fakeapi_native.cpp")]


def fakeapi_path() -> str:
    return os.path.join(ROOT, "ncc", "fakeapi", "_native" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_extension(debug: bool = False, sanitize: bool = False, verbose: bool = False, sources: list | None = None,
                    out: str | None = None) -> str:
    """A pybind11 extension: the product's `ncc._native` by default, or `sources` into `out`."""
    import pybind11

    out = out or target_path()
    sources = sources or SOURCES
    flavor = "sanitize" if sanitize else ("debug" if debug else "release")
    stamp = out + ".flavor"
    if flavor == "release" and os.path.exists(out) and os.path.exists(stamp):
        so_m = os.path.getmtime(out)
        with open(stamp) as f:
            same = f.read().strip() == flavor
        if same and all(os.path.getmtime(s) <= so_m for s in sources + COMMON_HEADERS + EXT_HEADERS + [__file__]):
            return out
    cxx = os.environ.get("CXX", "g++")
    flags = ["-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden", *arch_flags(), "-Wall", "-Wextra",
             "-Wno-unused-parameter"] + _werror()
    if debug or sanitize:
        flags += ["-O1", "-g", "-fno-omit-frame-pointer"]
    else:
        flags += ["-O3", "-DNDEBUG"]
    if sanitize:
        flags += ["-fsanitize=address,undefined"]
    incs = ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]
    tmp = out + ".tmp"
    cmd = [cxx, *flags, *incs, *sources, "-o", tmp]
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd))
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(flavor)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--sanitize", action="store_true")
    ap.add_argument("--product-only", action="store_true",
                    help="the controller's extension and executor only (the container image): no fake-apiserver "
                         "extension, no test tools")
    ap.add_argument("--executor-coverage", action="store_true",
                    help="rebuild only ncc/bin/ncc-executor with gcov instrumentation (scripts/cpp_coverage.py)")
    a = ap.parse_args()
    if a.executor_coverage:
        print(build_executor(coverage=True, verbose=True))
        sys.exit(0)
    print(build(a.debug, a.sanitize, verbose=True, substrate=not a.product_only))
    if not a.product_only:
        try:
            print(build_tools(verbose=True))
        except (subprocess.CalledProcessError, OSError) as e:  # a test tool: its tests skip without it
            print(f"warning: build/tools/ncc-h2probe was not built ({e})", file=sys.stderr)
        try:  # the frame-pointer executor for sampling profiles (scripts/box/run.sh sample)
            print(build_executor(profile=True))
        except (subprocess.CalledProcessError, OSError) as e:
            print(f"warning: the profiling executor was not built ({e})", file=sys.stderr)
    sys.exit(0)
