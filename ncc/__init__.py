"""ncc — multi-cluster Nexus configuration-sync controller (NexusAlgorithmTemplate / Workgroup fan-out).

A from-scratch re-design of SneaksAndData/nexus-configuration-controller: an asyncio control
plane with a C++ runtime extension (`ncc._native`) and an in-process fake kube-apiserver for
tests and benchmarks.  See README.md and SURVEY.md.
"""
__version__ = "0.1.0"
