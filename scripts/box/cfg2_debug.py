"""Box diagnostics for config 2's first-wave tail: run it with the controller's CPU/stats report and print
the controller log (executor enqueue causes, retries) plus per-wave timings."""
import asyncio
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "bench"))
os.environ["NCC_CPU_REPORT"] = "1"
import suite  # noqa: E402

orig = suite.Topology.stop


async def stop(self):
    for p in reversed(self.procs):
        if p.poll() is None:
            p.terminate()
    for p in self.procs:
        try:
            p.wait(timeout=15)
        except Exception:  # noqa: BLE001
            p.kill()
    with open(os.path.join(self.work, "controller.log"), errors="replace") as f:
        for line in f.read().splitlines()[-40:]:
            if "stats" in line or "report" in line or "rror" in line or "etry" in line:
                print(line[:600])
    await orig(self)

suite.Topology.stop = stop
r = asyncio.run(suite.config_cold_and_waves(2, 100, "native", waves=10, timeout=60, label="2"))
print(json.dumps(r)[:600])
