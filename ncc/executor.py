"""`python -m ncc.executor` — a shard-executor process (spawned by the coordinator; see ncc/controller/executor.py)."""
import sys

from .controller.executor import main

if __name__ == "__main__":
    sys.exit(main())
