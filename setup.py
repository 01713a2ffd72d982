"""Packaging hook for the C++ runtime extension `ncc._native` (sources in native/).

`pip install .` / `python -m build` compile it with the same flags as `python native/build.py`, which
remains the in-tree development build (it is what CI, `__graft_entry__.build()` and the tests use).
"""
from pybind11.setup_helpers import Pybind11Extension
from setuptools import setup

setup(ext_modules=[Pybind11Extension(
    "ncc._native", ["native/ncc_native.cpp"], cxx_std=17,
    extra_compile_args=["-O3", "-DNDEBUG", "-fvisibility=hidden", "-Wall", "-Wextra", "-Wno-unused-parameter"])])
