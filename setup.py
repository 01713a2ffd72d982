"""Packaging hook for the native code: the C++ runtime extension `ncc._native` (sources in native/), the fake
apiserver's `ncc.fakeapi._native` (native/fakeapi/) and the native shard executor `ncc/bin/ncc-executor`
(native/executor/, C++20 + OpenSSL).

`pip install .` / `python -m build` compile both with the same flags as `python native/build.py`, which
remains the in-tree development build (it is what CI, `__graft_entry__.build()` and the tests use).  The
executor needs g++ with C++20 coroutines and the OpenSSL headers (libssl-dev); without them the package
still installs and native mode runs the Python executor (`executor-impl: auto`).
"""
import os
import sys

from pybind11.setup_helpers import Pybind11Extension, build_ext
from setuptools import setup

HERE = os.path.dirname(os.path.abspath(__file__))


class BuildWithExecutor(build_ext):
    def run(self):
        super().run()
        sys.path.insert(0, os.path.join(HERE, "native"))
        import build as native_build  # native/build.py
        out = os.path.join(self.build_lib, "ncc", "bin", "ncc-executor")
        try:
            native_build.build_executor(out=out)
        except Exception as e:  # noqa: BLE001 — the Python executor remains
            print(f"warning: native shard executor not built ({e}); native mode will use the Python executor")


sys.path.insert(0, os.path.join(HERE, "native"))
from build import arch_flags  # noqa: E402 — native/build.py: -mpopcnt on x86-64 only

_FLAGS = ["-O3", "-DNDEBUG", "-fvisibility=hidden", *arch_flags(), "-Wall", "-Wextra", "-Wno-unused-parameter"]
# the controller's extension, and the fake apiserver's (ncc.fakeapi: test/bench substrate, kept out of the
# controller's .so — native/fakeapi/)
setup(ext_modules=[Pybind11Extension("ncc._native", ["native/ncc_native.cpp"], cxx_std=17, extra_compile_args=_FLAGS),
                   Pybind11Extension("ncc.fakeapi._native", ["native/fakeapi/fakeapi_native.cpp"], cxx_std=17,
                                     extra_compile_args=_FLAGS)],
      cmdclass={"build_ext": BuildWithExecutor})
