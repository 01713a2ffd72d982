"""Process resource limits for the long-running processes.

A native-mode controller keeps many sockets open: every shard executor holds up to 256 keep-alive
connections per shard plus its watch streams, and a fake apiserver in the benches serves all of them.
Many hosts start processes with a soft RLIMIT_NOFILE of 1024.  Like the Go runtime (which raises the
soft limit to the hard limit at start-up since Go 1.19, and so does the reference controller's
binary), every ncc process raises its soft file-descriptor limit to the hard limit.
"""
from __future__ import annotations


def raise_nofile_limit(cap: int = 1 << 20) -> int:
    """Raise the soft RLIMIT_NOFILE to the hard limit (at most `cap`); returns the soft limit in force."""
    try:
        import resource
        soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
        want = hard if hard != resource.RLIM_INFINITY else cap
        want = min(want, cap)
        if soft != resource.RLIM_INFINITY and soft < want:
            resource.setrlimit(resource.RLIMIT_NOFILE, (want, hard))
            return want
        return soft
    except (ImportError, ValueError, OSError):  # pragma: no cover - platform without rlimits
        return -1
