"""API layer: CRD contract constants, resource registry, object and reference helpers."""
from . import constants, objects, refs, resources  # noqa: F401
